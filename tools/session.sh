#!/bin/bash
# The current GPU-box session (rewritten per session; run through gpurun): every GPU step under its own time limit,
# stop at the first failure.
set -u
export TMPDIR=/tmp
R=$(pwd); OUT=$R/gpurun_out; mkdir -p "$OUT"
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "== $name $(date +%T)" | tee -a "$OUT/steps.log"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc" | tee -a "$OUT/steps.log"
  return $rc
}
step pytest 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider || exit $?
AB_REPS=3 step ab 900 bash tools/ab_bench_libs.sh librtc.so librtc_grp0.so librtc_grp_accb0.so || exit $?
cd /tmp
step loop1 120 rocprofv3 --kernel-trace --stats -d "$OUT/loop1" -o run --output-format csv -- python3 "$R/tools/frame_loop.py" 40 overlap 1 || exit $?
echo done
