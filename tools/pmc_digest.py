#!/usr/bin/env python3
"""Roofline inputs of one workload from its rocprofv3 runs (tools/profile_workload.sh) -> profiles/pmc_<workload>.json,
which bench.py reads for roofline.kernels.  Not part of the product.

Per kernel: the kernel-trace average duration (rocprofv3 --kernel-trace --stats of the bench command, kernels running
concurrently as in the timed frames) and, from the PMC passes over tools/one_render.py <workload> (one counter group
per run), the counters per dispatch.  The kernel with the longest isolated dispatch (the critical path) is named
`dominant`.

HBM bytes (MI355X_MICROARCH.md, HBM section): WRITE_SIZE is exact for 16-B-per-lane streaming stores and taken as is;
FETCH_SIZE reads half the bytes of WIDE COALESCED STREAMING reads (16 B/lane) only.  This path's reads are small
gathers (scene records staged once per workgroup, 12-B sample slots, 4-B list entries), so FETCH_SIZE is used raw and
calibrated on rtc_accumulate_samples, whose read bytes are known exactly (items x spp x 12 B + 4 B per item): the
calibration factor is reported, not applied.  Usage: pmc_digest.py <profile dir> <workload> [items]"""
import collections
import csv
import glob
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
root, workload = sys.argv[1], sys.argv[2]
KERNELS = ("rtc_render_chain", "rtc_render_sky", "rtc_accumulate_samples", "rtc_tile_cull", "rtc_super_cull",
           "rtc_prep_primary")


def short(name):
    for k in KERNELS:
        if k in name:
            return k
    return None


# kernel trace stats
stats = {}
for f in glob.glob(os.path.join(root, "trace", "**", "*kernel_stats.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        k = short(r["Name"])
        # the timed instantiation: rtc_render_chain<MULTI, COUNT=false>; the counting one runs only for the counters
        if k and not r["Name"].endswith("true>(RenderParams)"):
            stats[k] = {"calls": int(r["Calls"]), "avg_ms": float(r["AverageNs"]) / 1e6,
                        "total_ms": float(r["TotalDurationNs"]) / 1e6}
# counters: every pass directory pmc_* holds one counter group over the same renders
per = collections.defaultdict(dict)
for d in sorted(glob.glob(os.path.join(root, "pmc_*"))):
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        acc = collections.defaultdict(lambda: collections.defaultdict(float))
        for r in csv.DictReader(open(f)):
            k = short(r.get("Kernel_Name", ""))
            if k and not r.get("Kernel_Name", "").endswith("true>(RenderParams)"):
                acc[k][(r["Counter_Name"], r.get("Dispatch_Id"))] += float(r["Counter_Value"])
        for k, cv in acc.items():
            by = collections.defaultdict(list)
            for (c, _), v in cv.items():
                by[c].append(v)
            for c, vs in by.items():  # per dispatch: the mean over this pass's dispatches
                per[k][c] = sum(vs) / len(vs)
out = {"workload": workload, "n_gpus": 1,
       "source": f"rocprofv3 kernel trace of bench.py --workload {workload} + PMC passes over tools/one_render.py "
                 f"{workload} (profiles/pmc_{workload}.json, tools/pmc_digest.py)",
       "kernels": {}}
for k in KERNELS:
    if k not in per and k not in stats:
        continue
    pd = {c: round(v, 1) for c, v in sorted(per.get(k, {}).items())}
    e = {"per_dispatch": pd}
    if k in stats:
        e["rocprof_avg_ms"] = round(stats[k]["avg_ms"], 5)
        e["rocprof_total_ms"] = round(stats[k]["total_ms"], 3)
        e["rocprof_calls"] = stats[k]["calls"]
    if "FETCH_SIZE" in pd or "WRITE_SIZE" in pd:
        fb = pd.get("FETCH_SIZE", 0.0) * 1024
        wb = pd.get("WRITE_SIZE", 0.0) * 1024
        e["fetch_bytes_raw"] = int(fb)
        e["write_bytes"] = int(wb)
        e["traffic_bytes"] = int(fb + wb)
        e["traffic_note"] = "FETCH_SIZE raw + WRITE_SIZE (KB x 1024); no x2: these reads are not 16-B streaming reads"
    out["kernels"][k] = e
if len(sys.argv) > 3:  # calibration on the accumulate pass: its read bytes are known
    items = int(sys.argv[3])
    spp = {"ultracomplex_1080p64": 64, "ultracomplex_4k64": 64, "ultracomplex_4k256": 256, "complex_4k64": 64,
           "fsuzane_1080p64": 64, "cube_1080p16": 16, "simplest_256p1": 1}[workload]
    acc = out["kernels"].get("rtc_accumulate_samples", {})
    if acc.get("fetch_bytes_raw"):
        known = items * (spp * 12 + 4)
        out["fetch_calibration"] = {"kernel": "rtc_accumulate_samples", "known_read_bytes": known,
                                    "fetch_bytes_raw": acc["fetch_bytes_raw"],
                                    "raw_over_known": round(acc["fetch_bytes_raw"] / known, 4)}
if stats:
    # the critical-path kernel: the longest dispatch when it runs alone (GRBM_GUI_ACTIVE of the PMC pass; the chain and
    # sky kernels run concurrently in the frame, and their rocprof totals are within 1 % of each other on the BASELINE
    # frame, which made a total-time choice flip from box to box)
    def isolated(k):
        pd = (out.get("kernels", {}).get(k) or {}).get("per_dispatch") or {}
        return (pd.get("GRBM_GUI_ACTIVE") or 0, stats[k]["total_ms"])
    out["dominant"] = max((k for k in stats if k in ("rtc_render_chain", "rtc_render_sky")), key=isolated, default=None)
path = os.path.join(REPO, "profiles", f"pmc_{workload}.json")
json.dump(out, open(path, "w"), indent=1)
print(json.dumps(out, indent=1))
