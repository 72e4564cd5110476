#!/bin/bash
# bench.py headline for library variants, alternating (two rounds): tools/ab_bench_libs.sh [--workload w] lib1.so lib2.so ...
set -u
wl=ultracomplex_1080p64
if [ "${1:-}" = "--workload" ]; then wl=$2; shift 2; fi
for rep in $(seq 1 ${AB_REPS:-2}); do
  for l in "$@"; do
    RTC_LIB_PATH=$GRAFT_REPO_ROOT/raytracingc_amd/_lib/$l timeout -k 10 200 python bench.py --workload $wl --steps 50 --warmup 5 \
      --no-extras --no-cpu-baseline > gpurun_out/abl.log 2>&1 || { echo "$l failed"; exit 1; }
    python3 - "$l" <<'P'
import json, sys
d = json.loads([l for l in open("gpurun_out/abl.log") if l.startswith("{")][-1])
k = d["roofline"]["kernels"]
print(sys.argv[1], d["config"]["workload"], "frame", d["ms_per_step"], "chain", k["rtc_render_chain"]["ms"], "sky", k["rtc_render_sky"]["ms"])
P
  done
done
