#!/bin/bash
# bench.py headline for library variants, alternating (two rounds): tools/ab_bench_libs.sh lib1.so lib2.so ...
set -u
for rep in 1 2; do
  for l in "$@"; do
    RTC_LIB_PATH=$GRAFT_REPO_ROOT/raytracingc_amd/_lib/$l timeout -k 10 200 python bench.py --steps 50 --warmup 5 \
      --no-extras --no-cpu-baseline > gpurun_out/abl.log 2>&1 || { echo "$l failed"; exit 1; }
    echo "$l $(tail -1 gpurun_out/abl.log | grep -o '"ms_per_step": [0-9.]*')"
  done
done
