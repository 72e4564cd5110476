#!/bin/bash
# One GPU-box session for this round: parity tests, smoke, bench (and optional extra commands).  Each GPU step
# has its own time limit; the script stops at the first failure.  usage: tools/gpu_session.sh [tests|bench|all]
set -u
export TMPDIR=/tmp
R=$(pwd)
OUT=$R/gpurun_out
mkdir -p "$OUT"
what=${1:-all}
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "== $name $(date +%T)" | tee -a "$OUT/steps.log"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc" | tee -a "$OUT/steps.log"
  tail -5 "$OUT/$name.log"
  return $rc
}
if [ "$what" = all ] || [ "$what" = tests ]; then
  step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v -s --timeout 180 --timeout-method thread -p no:cacheprovider || exit $?
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
fi
if [ "$what" = all ] || [ "$what" = bench ]; then
  step bench 600 python bench.py --steps 20 --warmup 3 || exit $?
fi
echo done
