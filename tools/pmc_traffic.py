#!/usr/bin/env python3
"""HBM traffic per launch of the split launch's kernels from the rocprofv3 FETCH_SIZE / WRITE_SIZE passes of
tools/round_gpu.sh (gpurun_out/pmc_fetch, gpurun_out/pmc_write) -> profiles/pmc_traffic.json, which bench.py
reads for roofline.traffic.  Not part of the product.

Corrections (MI355X_MICROARCH.md, HBM section): both counters are in KB; on gfx950 FETCH_SIZE reports half
the bytes of wide coalesced reads, so it is doubled; WRITE_SIZE is taken as is.  The render kernels' reads
are small (scene records, staged once per workgroup into LDS) and their writes are the 3-byte pixels, so the
absolute numbers are indicative only (other access widths are uncalibrated per the guide).
Usage: pmc_traffic.py [gpurun_out] [workload]"""
import collections
import csv
import glob
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
root = sys.argv[1] if len(sys.argv) > 1 else os.path.join(REPO, "gpurun_out")
workload = sys.argv[2] if len(sys.argv) > 2 else "ultracomplex_1080p64"


def per_kernel(pass_dir, counter):
    vals = collections.defaultdict(list)
    for f in glob.glob(os.path.join(root, pass_dir, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            rows = list(csv.DictReader(fh))
        acc = collections.defaultdict(float)
        for r in rows:
            if r["Counter_Name"] == counter:
                acc[(r["Kernel_Name"].split("(")[0], r.get("Dispatch_Id"))] += float(r["Counter_Value"])
        for (k, _), v in acc.items():
            vals[k].append(v)
    return vals


fetch = per_kernel("pmc_fetch", "FETCH_SIZE")
write = per_kernel("pmc_write", "WRITE_SIZE")
out = {}
path = os.path.join(REPO, "profiles", "pmc_traffic.json")
if os.path.exists(path):
    out = json.load(open(path))
entry = {"n_gpus": 1, "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over tools/one_render.py faithful",
         "kernels": {}}
for k in sorted(set(fetch) | set(write)):
    if not any(s in k for s in ("rtc_render_heavy", "rtc_render_chain", "rtc_render_sky", "rtc_tile_cull",
                                "rtc_prep_primary", "rtc_order_heavy", "rtc_pixel_list", "rtc_reduce_segments")):
        continue
    f = fetch.get(k, [])
    w = write.get(k, [])
    fk = sum(f) / len(f) if f else 0.0
    wk = sum(w) / len(w) if w else 0.0
    entry["kernels"][k] = {"fetch_kb_raw": round(fk, 3), "write_kb": round(wk, 3), "dispatches": max(len(f), len(w)),
                           "hbm_bytes_per_launch": int(2 * fk * 1024 + wk * 1024)}
for name in ("rtc_render_chain", "rtc_render_heavy"):  # the split launch's heavy-tile kernel
    heavy = [v for k, v in entry["kernels"].items() if name in k]
    if heavy:
        entry["kernel"] = name
        entry["hbm_bytes_per_launch"] = heavy[0]["hbm_bytes_per_launch"]
        break
out[workload] = entry
os.makedirs(os.path.dirname(path), exist_ok=True)
json.dump(out, open(path, "w"), indent=1)
print(json.dumps(out, indent=1))
