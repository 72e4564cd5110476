#!/bin/bash
# bench.py's headline (frame incl. pipelined D2H) for D2H methods, alternating: tools/ab_d2h_blocks.sh 0 16 32 ...
set -u
for rep in 1 2 3; do
  for n in "$@"; do
    timeout -k 10 200 python bench.py --steps 60 --warmup 5 --no-extras --no-cpu-baseline --d2h-blocks $n > gpurun_out/abd_$n.log 2>&1 || { echo "$n failed"; tail -3 gpurun_out/abd_$n.log; exit 1; }
    tail -1 gpurun_out/abd_$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n', d['ms_per_step'], 'd2h', d['d2h_ms'], 'dev', d['device_only']['ms_per_step'] if 'device_only' in d else None, d['host_frame_equals_device_frame'])"
  done
done
