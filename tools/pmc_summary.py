#!/usr/bin/env python3
"""Summarise rocprofv3 counter CSVs (tools/pmc_breakdown.sh output) per kernel: counter totals over the
kernel's dispatches, and a few derived ratios.  Not part of the product.
Usage: pmc_summary.py <dir> [kernel-substring ...]"""
import collections
import csv
import glob
import json
import os
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmcb"
kernels = sys.argv[2:] or ["rtc_render_chain", "rtc_render_heavy", "rtc_render_sky", "rtc_tile_cull"]
tot = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    with open(f) as fh:
        for row in csv.DictReader(fh):
            name = row.get("Kernel_Name", "")
            for k in kernels:
                if k in name:
                    tot[k][row["Counter_Name"]] += float(row["Counter_Value"])
                    disp[k].add((f, row.get("Dispatch_Id")))
out = {}
for k in kernels:
    c = tot[k]
    d = dict(sorted(c.items()))
    valu = c.get("SQ_INSTS_VALU", 0)
    if valu:
        d["_valu_per_wave"] = valu / max(c.get("SQ_WAVES", 1), 1)
        f64 = sum(c.get(x, 0) for x in ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64",
                                         "SQ_INSTS_VALU_TRANS_F64"))
        d["_f64_share_of_valu"] = f64 / valu
    if c.get("SQ_WAVE_CYCLES"):
        d["_active_valu_over_wave_cycles"] = c.get("SQ_ACTIVE_INST_VALU", 0) / c["SQ_WAVE_CYCLES"]
        d["_wait_inst_any_over_wave_cycles"] = c.get("SQ_WAIT_INST_ANY", 0) / c["SQ_WAVE_CYCLES"]
    # dispatches per counter pass (each pass is its own run over the same renders; counters of one pass are
    # totals over that pass's dispatches)
    per_file = collections.Counter(f for f, _ in disp[k])
    n = max(per_file.values()) if per_file else 0
    d["_dispatches_per_pass"] = n
    if n:
        d["_per_dispatch"] = {c: v / n for c, v in sorted(c.items())}
    out[k] = d
print(json.dumps(out, indent=1))
