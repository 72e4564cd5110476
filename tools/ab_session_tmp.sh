set -u
export TMPDIR=/tmp
R=$(pwd); mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r04_c.log 2>&1 || { echo tests failed; tail -30 gpurun_out/pytest_r04_c.log; exit 1; }
tail -2 gpurun_out/pytest_r04_c.log
AB_REPS=2 timeout -k 10 600 bash tools/ab_bench_libs.sh librtc_new.so librtc_oldbm.so librtc_sky8.so librtc_sky7.so > gpurun_out/ab_r04_c.log 2>&1 || { echo ab failed; cat gpurun_out/ab_r04_c.log; exit 1; }
cat gpurun_out/ab_r04_c.log
timeout -k 10 200 python tools/scale_probe.py 5 1920 1080 64 overlap > gpurun_out/scale1080_r04_c.log 2>&1 || exit 1
cat gpurun_out/scale1080_r04_c.log
