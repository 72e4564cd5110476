#!/bin/bash
# GPU-box check: parity tests, smoke, a short bench and a rocprofv3 kernel-trace summary.
# Every GPU step has its own time limit; the script stops at the first crash / timeout (rc >= 2).
set -u
export TMPDIR=/tmp
R=$(pwd)
OUT=$R/gpurun_out
mkdir -p "$OUT"
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "== $name" | tee -a "$OUT/steps.log"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc" | tee -a "$OUT/steps.log"
  tail -3 "$OUT/$name.log"
  return $rc
}
lim=${1:-all}
step pytest_gpu 900 python -m pytest tests -m gpu -q -s -p no:cacheprovider; rc=$?
[ $rc -le 1 ] || exit $rc
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
[ "$lim" = "tests" ] && exit 0
step bench 600 python bench.py --steps 5 --warmup 2 || exit $?
cd /tmp && step rocprof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu-baseline --no-hoisted || exit $?
echo done
