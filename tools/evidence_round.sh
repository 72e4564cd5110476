#!/bin/bash
# Round evidence: GPU tests + smoke, the bench line (with CPU baseline), the other BASELINE configs, rocprofv3
# kernel-trace + PMC passes, rank-share scale probes, an overlapped frame-loop trace.  Each GPU step has its own
# time limit; the script stops at the first failing step.  usage: tools/evidence_round.sh <tag>
set -u
export TMPDIR=/tmp
R=$(pwd); OUT=$R/gpurun_out; tag=${1:-r02_e}
mkdir -p "$OUT"
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "== $name $(date +%T)" | tee -a "$OUT/steps.log"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc" | tee -a "$OUT/steps.log"
  return $rc
}
step "pytest_$tag" 400 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread -p no:cacheprovider || exit $?
step "smoke_$tag" 200 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
step "bench_$tag" 500 python bench.py --steps 30 --warmup 5 || exit $?
for w in ultracomplex_4k64 complex_4k64 ultracomplex_4k256 fsuzane_1080p64 cube_1080p16 simplest_256p1; do
  step "bench_${tag}_$w" 300 python bench.py --workload $w --steps 10 --warmup 3 --no-extras --no-cpu-baseline || exit $?
done
step "scale1080_$tag" 200 python tools/scale_probe.py 7 || exit $?
step "scale4k_$tag" 200 python tools/scale_probe.py 5 3840 2160 64 || exit $?
bash tools/prof_session.sh "$tag" || exit $?
cd /tmp
step "loop_$tag" 200 rocprofv3 --kernel-trace --stats -d "$OUT/loop_$tag" -o run --output-format csv -- python3 "$R/tools/frame_loop.py" 40 overlap || exit $?
echo done
