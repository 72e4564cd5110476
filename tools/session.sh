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
tag=${1:-r03_c}
step pytest_$tag 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider || exit $?
step smoke_$tag 200 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
step bench_$tag 400 python bench.py || exit $?
step scale1080_$tag 200 python tools/scale_probe.py 5 1920 1080 64 overlap || exit $?
step scale4k_$tag 200 python tools/scale_probe.py 5 3840 2160 64 overlap || exit $?
bash tools/profile_workload.sh ultracomplex_1080p64 $tag || exit $?
echo done
