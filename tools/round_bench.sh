#!/bin/bash
# Bench lines for the headline workload and every other BASELINE config (1 GPU), each under its own time limit.
set -u
R=$(pwd); OUT=$R/gpurun_out; tag=${1:-r02}
mkdir -p "$OUT"
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > "$OUT/bench_${tag}.log" 2>&1 || exit $?
tail -1 "$OUT/bench_${tag}.log"
for w in ultracomplex_4k64 complex_4k64 ultracomplex_4k256 fsuzane_1080p64 cube_1080p16 simplest_256p1; do
  timeout -k 10 300 python bench.py --workload $w --steps 10 --warmup 3 --no-extras --no-cpu-baseline > "$OUT/bench_${tag}_$w.log" 2>&1 || exit $?
  tail -1 "$OUT/bench_${tag}_$w.log" | cut -c1-400
done
