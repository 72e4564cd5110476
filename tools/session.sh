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
step bench1 150 python bench.py --steps 50 --warmup 5 --no-cpu-baseline || exit $?
step one_chain 100 python tools/one_render.py ultracomplex_1080p64 5 || exit $?
step sections 200 python tools/chain_sections.py || exit $?
bash tools/profile_workload.sh ultracomplex_1080p64 r03a || exit $?
echo done
