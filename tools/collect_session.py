#!/usr/bin/env python3
"""Copy a tools/session.sh run's outputs from gpurun_out/ into profiles/ under its tag (bench lines as JSON, logs,
the rocprofv3 kernel stats, the raw PMC CSVs, rank shares, rehearsals, frame-loop stats).  Not part of the product.
Usage: collect_session.py <tag>"""
import glob
import json
import os
import shutil
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
G, P = os.path.join(REPO, "gpurun_out"), os.path.join(REPO, "profiles")
tag = sys.argv[1]


def jline(src, dst):
    if not os.path.exists(src):
        return
    lines = [x for x in open(src) if x.startswith("{")]
    if lines:
        json.dump(json.loads(lines[-1]), open(dst, "w"), indent=1)
        print("wrote", os.path.relpath(dst, REPO))


jline(f"{G}/bench_{tag}.log", f"{P}/{tag}_bench.json")
for f in glob.glob(f"{G}/bench_{tag}_*.log"):
    w = os.path.basename(f)[len(f"bench_{tag}_"):-4]
    jline(f, f"{P}/{tag}_bench_{w}.json")
for src, dst in ((f"pytest_{tag}.log", f"{tag}_pytest_gpu.log"), (f"smoke_{tag}.log", f"{tag}_smoke.log"),
                 (f"sections_{tag}.log", f"{tag}_chain_sections.log")):
    if os.path.exists(f"{G}/{src}"):
        shutil.copy(f"{G}/{src}", f"{P}/{dst}")
        print("wrote", dst)
scales = [n for n in (f"scale1080_{tag}", f"scale1080_band8_{tag}", f"scale4k_{tag}", f"scale4k_band8_{tag}")
          if os.path.exists(f"{G}/{n}.log")]
if scales:
    with open(f"{P}/{tag}_rank_share_overlap.log", "w") as f:
        for n in scales:
            f.write(f"# tools/scale_probe.py ({n})\n" + "".join(x for x in open(f"{G}/{n}.log") if x.startswith("{")))
    print("wrote", f"{tag}_rank_share_overlap.log")
for n, t in ((f"rehearse2_{tag}", "rehearsal_n2_gloo_one_gpu"), (f"rehearse8_{tag}", "rehearsal_n8_gloo_one_gpu"),
             (f"rehearse8_band8_{tag}", "rehearsal_n8_band8_gloo_one_gpu")):
    jline(f"{G}/{n}.log", f"{P}/{tag}_{t}.json")
for n, t in ((f"loop1_{tag}", "frame_loop_n1_kernel_stats.csv"), (f"loop8_{tag}", "frame_loop_share8_kernel_stats.csv")):
    if os.path.exists(f"{G}/{n}/run_kernel_stats.csv"):
        shutil.copy(f"{G}/{n}/run_kernel_stats.csv", f"{P}/{tag}_{t}")
        print("wrote", f"{tag}_{t}")
d = f"{G}/prof_ultracomplex_1080p64_{tag}"
if os.path.isdir(d):
    os.makedirs(f"{P}/{tag}_pmc", exist_ok=True)
    for g in range(1, 6):
        for f in glob.glob(f"{d}/pmc_g{g}/**/*counter_collection.csv", recursive=True):
            shutil.copy(f, f"{P}/{tag}_pmc/pmc_g{g}_counter_collection.csv")
    for f in glob.glob(f"{d}/trace/**/*kernel_stats.csv", recursive=True):
        shutil.copy(f, f"{P}/{tag}_rocprof_kernel_stats.csv")
    if os.path.exists(f"{G}/pmc_ultracomplex_1080p64.json"):
        shutil.copy(f"{G}/pmc_ultracomplex_1080p64.json", f"{P}/pmc_ultracomplex_1080p64.json")
    print("wrote", f"{tag}_pmc/, {tag}_rocprof_kernel_stats.csv, pmc_ultracomplex_1080p64.json")
