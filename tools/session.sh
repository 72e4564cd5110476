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
for w in ultracomplex_1080p64 ultracomplex_4k64 fsuzane_1080p64; do
  for lib in librtc.so librtc_waves5.so librtc_waves5s.so; do
    RTC_LIB_PATH=$R/raytracingc_amd/_lib/$lib step "ab_${w}_${lib%.so}" 150 python bench.py --workload $w --steps 30 --warmup 5 --no-cpu-baseline --no-extras || exit $?
  done
done
step scale1080 200 python tools/scale_probe.py 5 1920 1080 64 overlap || exit $?
cd /tmp
step loop8 120 rocprofv3 --kernel-trace --stats -d "$OUT/loop8" -o run --output-format csv -- python3 "$R/tools/frame_loop.py" 60 overlap 8 || exit $?
step loop1 120 rocprofv3 --kernel-trace --stats -d "$OUT/loop1" -o run --output-format csv -- python3 "$R/tools/frame_loop.py" 40 overlap 1 || exit $?
echo done
