set -u
export TMPDIR=/tmp
R=$(pwd); mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_head.log 2>&1 || { echo pytest head failed; tail -30 gpurun_out/pytest_head.log; exit 1; }
echo "head: $(tail -1 gpurun_out/pytest_head.log)"
RTC_LIB_PATH=$R/raytracingc_amd/_lib/librtc_new2.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_new.log 2>&1 || { echo pytest failed; tail -30 gpurun_out/pytest_new.log; exit 1; }
echo "new2: $(tail -1 gpurun_out/pytest_new.log)"
AB_REPS=3 timeout -k 10 400 bash tools/ab_bench_libs.sh librtc_cur.so librtc_new.so librtc_new2.so > gpurun_out/ab_new.log 2>&1 || { echo ab failed; cat gpurun_out/ab_new.log; exit 1; }
cat gpurun_out/ab_new.log
SCALE_NS=8,4 timeout -k 10 400 bash tools/ab_scale.sh overlap librtc_cur.so librtc_new.so librtc_new2.so > gpurun_out/abs_new.log 2>&1 || { cat gpurun_out/abs_new.log; exit 1; }
cat gpurun_out/abs_new.log
