#!/usr/bin/env python3
"""Static instruction counts of one kernel's ISA between s_memtime / s_memrealtime markers (the RTC_DIAG
build's section timers), by class.  Not part of the product.
Usage: isa_sections.py <file.s> <mangled-kernel-name>"""
import re
import sys

path, name = sys.argv[1], sys.argv[2]
text = open(path).read().split("\n")
body, on = [], False
for line in text:
    if line.startswith(name + ":"):
        on = True
        continue
    if on and line.startswith(".Lfunc_end"):
        break
    if on:
        body.append(line.strip())
segs, cur = [], []
for t in body:
    if not t or t.startswith(";") or (t.startswith(".") and not t.startswith(".LBB")):
        continue
    if "s_memtime" in t or "s_memrealtime" in t:
        segs.append(cur)
        cur = []
        continue
    cur.append(t)
segs.append(cur)
tot = [0, 0, 0, 0, 0]
for i, sg in enumerate(segs):
    v = sum(1 for t in sg if t.startswith("v_"))
    d = sum(1 for t in sg if re.match(r"v_\w+_f64", t))
    s = sum(1 for t in sg if t.startswith("s_"))
    ds = sum(1 for t in sg if t.startswith("ds_"))
    tot = [a + b for a, b in zip(tot, [len(sg), v, d, s, ds])]
    first = next((t for t in sg if not t.startswith(".LBB")), "")
    print(f"{i:3d} lines {len(sg):5d} valu {v:5d} f64 {d:4d} salu {s:5d} lds {ds:4d}   {first[:60]}")
print("total lines %d valu %d f64 %d salu %d lds %d" % tuple(tot))
if len(sys.argv) > 3:  # opcode histograms of the listed sections
    import collections
    for i in (int(x) for x in sys.argv[3].split(",")):
        c = collections.Counter(t.split()[0] for t in segs[i] if not t.startswith(".LBB"))
        print(i, c.most_common(30))
