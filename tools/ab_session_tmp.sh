set -u
export TMPDIR=/tmp
R=$(pwd); mkdir -p gpurun_out
# parity of the candidate first (the whole GPU suite through the variant library)
RTC_LIB_PATH=$R/raytracingc_amd/_lib/librtc_pu2.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_pu2.log 2>&1 || { echo pytest failed; tail -30 gpurun_out/pytest_pu2.log; exit 1; }
tail -2 gpurun_out/pytest_pu2.log
AB_REPS=2 timeout -k 10 500 bash tools/ab_bench_libs.sh librtc_old.so librtc_pu.so librtc_pu2.so > gpurun_out/ab_pow.log 2>&1 || { echo ab failed; cat gpurun_out/ab_pow.log; exit 1; }
cat gpurun_out/ab_pow.log
AB_REPS=1 timeout -k 10 300 bash tools/ab_bench_libs.sh --workload fsuzane_1080p64 librtc_old.so librtc_pu2.so > gpurun_out/ab_pow_fs.log 2>&1 || { echo ab failed; cat gpurun_out/ab_pow_fs.log; exit 1; }
cat gpurun_out/ab_pow_fs.log
SCALE_NS=8 timeout -k 10 300 bash tools/ab_scale.sh overlap librtc_old.so librtc_pu2.so > gpurun_out/abs_pow.log 2>&1 || { cat gpurun_out/abs_pow.log; exit 1; }
cat gpurun_out/abs_pow.log
