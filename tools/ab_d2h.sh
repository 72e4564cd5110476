#!/bin/bash
# bench.py's headline (frame incl. pipelined D2H) per D2H method, alternating: tools/ab_d2h_blocks.sh dma kernel runtime
set -u
for rep in 1 2 3; do
  for m in "$@"; do
    timeout -k 10 200 python bench.py --steps 60 --warmup 5 --no-cpu-baseline --d2h $m > gpurun_out/abd_$m.log 2>&1 || { echo "$m failed"; tail -3 gpurun_out/abd_$m.log; exit 1; }
    tail -1 gpurun_out/abd_$m.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$m', d['ms_per_step'], 'd2h', d['d2h_ms'], 'dev', d['device_only']['ms_per_step'], 'lat', d['frame_latency_ms'], d['host_frame_equals_device_frame'])"
  done
done
