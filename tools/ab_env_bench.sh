#!/bin/bash
# bench.py's headline (frame incl. pipelined D2H) under DEBUG_CLR_LIMIT_BLIT_WG values, alternating.
set -u
for rep in 1 2 3; do
  for n in "$@"; do
    if [ "$n" = default ]; then unset DEBUG_CLR_LIMIT_BLIT_WG; else export DEBUG_CLR_LIMIT_BLIT_WG=$n; fi
    timeout -k 10 200 python bench.py --steps 60 --warmup 5 --no-extras --no-cpu-baseline > gpurun_out/abe_$n.log 2>&1 || { echo "$n failed"; exit 1; }
    tail -1 gpurun_out/abe_$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n', d['ms_per_step'], 'd2h', d['d2h_ms'])"
  done
done
