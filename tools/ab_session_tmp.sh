set -u
export TMPDIR=/tmp
R=$(pwd); mkdir -p gpurun_out
for v in cb128; do
RTC_LIB_PATH=$R/raytracingc_amd/_lib/librtc_$v.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_$v.log 2>&1 || { echo pytest $v failed; tail -30 gpurun_out/pytest_$v.log; exit 1; }
echo "$v: $(tail -1 gpurun_out/pytest_$v.log)"
done
AB_REPS=3 timeout -k 10 400 bash tools/ab_bench_libs.sh librtc_cur.so librtc_cb128.so > gpurun_out/ab_cb.log 2>&1 || { echo ab failed; cat gpurun_out/ab_cb.log; exit 1; }
cat gpurun_out/ab_cb.log
AB_REPS=1 timeout -k 10 300 bash tools/ab_bench_libs.sh --workload fsuzane_1080p64 librtc_cur.so librtc_cb128.so > gpurun_out/ab_cb_fs.log 2>&1 || { echo ab failed; cat gpurun_out/ab_cb_fs.log; exit 1; }
cat gpurun_out/ab_cb_fs.log
SCALE_NS=8,4 timeout -k 10 400 bash tools/ab_scale.sh overlap librtc_cur.so librtc_cb128.so > gpurun_out/abs_cb.log 2>&1 || { cat gpurun_out/abs_cb.log; exit 1; }
cat gpurun_out/abs_cb.log
