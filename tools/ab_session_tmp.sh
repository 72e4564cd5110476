set -u
export TMPDIR=/tmp
R=$(pwd); mkdir -p gpurun_out
RTC_LIB_PATH=$R/raytracingc_amd/_lib/librtc_nt.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_nt.log 2>&1 || { echo pytest failed; tail -30 gpurun_out/pytest_nt.log; exit 1; }
tail -2 gpurun_out/pytest_nt.log
AB_REPS=3 timeout -k 10 400 bash tools/ab_bench_libs.sh librtc_pu2.so librtc_nt.so librtc_ntu1.so librtc_ntu4.so > gpurun_out/ab_nt.log 2>&1 || { echo ab failed; cat gpurun_out/ab_nt.log; exit 1; }
cat gpurun_out/ab_nt.log
