#!/usr/bin/env python3
"""SGPR spill traffic (v_writelane / v_readlane) of one kernel by basic block and loop depth, from `hipcc -S` output.
Not part of the product.  Usage: spill_map.py <file.s> <mangled-kernel-name> [min-per-block]"""
import re
import sys

path, name = sys.argv[1], sys.argv[2]
mn = int(sys.argv[3]) if len(sys.argv) > 3 else 3
lines = open(path).read().split("\n")
on, cur, order, blocks = False, "entry", [("entry", "")], {"entry": []}
for l in lines:
    if l.startswith(name + ":"):
        on = True
        continue
    if on and l.startswith(".Lfunc_end"):
        break
    if not on:
        continue
    m = re.match(r"^(\.LBB\d+_\d+):(.*)", l)
    if m:
        cur = m.group(1)
        order.append((cur, m.group(2).strip()))
        blocks[cur] = []
    else:
        blocks[cur].append(l.strip())
bydepth = {}
for b, c in order:
    ins = [x for x in blocks[b] if x and not x.startswith((";", "."))]
    w = sum(x.startswith("v_writelane") for x in ins)
    r = sum(x.startswith("v_readlane") for x in ins)
    d = int(re.search(r"Depth=(\d+)", c).group(1)) if "Depth=" in c else 0
    bw, br = bydepth.get(d, (0, 0))
    bydepth[d] = (bw + w, br + r)
    if w + r >= mn:
        print(f"{b:12s} depth {d} insts {len(ins):4d} writelane {w:3d} readlane {r:3d}")
for d in sorted(bydepth):
    print(f"depth {d}: writelane {bydepth[d][0]} readlane {bydepth[d][1]}")
