set -u
export TMPDIR=/tmp
R=$(pwd); mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r04_h.log 2>&1 || { echo tests failed; tail -30 gpurun_out/pytest_r04_h.log; exit 1; }
tail -2 gpurun_out/pytest_r04_h.log
AB_REPS=2 timeout -k 10 500 bash tools/ab_bench_libs.sh librtc_new.so librtc_newinl.so > gpurun_out/ab_r04_h.log 2>&1 || { echo ab failed; cat gpurun_out/ab_r04_h.log; exit 1; }
for w in ultracomplex_4k64 fsuzane_1080p64 complex_4k64; do AB_REPS=1 timeout -k 10 500 bash tools/ab_bench_libs.sh --workload $w librtc_new.so librtc_newinl.so >> gpurun_out/ab_r04_h.log 2>&1 || exit 1; done
cat gpurun_out/ab_r04_h.log
SCALE_NS=8 timeout -k 10 400 bash tools/ab_scale.sh overlap librtc_new.so librtc_share3.so librtc_new.so librtc_share3.so > gpurun_out/abs_r04_h.log 2>&1 || { cat gpurun_out/abs_r04_h.log; exit 1; }
cat gpurun_out/abs_r04_h.log
