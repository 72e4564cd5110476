#!/bin/bash
# bench.py's headline (frame incl. pipelined D2H) for library variants, alternating: tools/ab_bench.sh lib1.so lib2.so ...
set -u
for rep in 1 2; do
  for lib in "$@"; do
    RTC_LIB_PATH=$PWD/raytracingc_amd/_lib/$lib timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-extras \
      --no-cpu-baseline > gpurun_out/abb_$lib.log 2>&1 || { echo "$lib failed"; tail -3 gpurun_out/abb_$lib.log; exit 1; }
    tail -1 gpurun_out/abb_$lib.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib', d['ms_per_step'], 'chain', d['roofline']['kernel_ms'], 'sky', d['roofline']['sky_kernel_ms'])"
  done
done
