#!/bin/bash
# host enqueue cost vs device period (tools/enqueue_probe.py) and the side stream's priority A/B (not part of the product)
set -u
R=$(pwd); OUT=$R/gpurun_out; mkdir -p "$OUT"
timeout -k 10 200 python tools/enqueue_probe.py > "$OUT/enqueue_o.log" 2>&1 || { tail -5 "$OUT/enqueue_o.log"; exit 1; }
grep '^{' "$OUT/enqueue_o.log"
AB_REPS=2 bash tools/ab_session.sh o librtc.so librtc_sidehi.so
