set -u
export TMPDIR=/tmp
R=$(pwd); mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r04_i.log 2>&1 || { echo tests failed; tail -30 gpurun_out/pytest_r04_i.log; exit 1; }
tail -2 gpurun_out/pytest_r04_i.log
timeout -k 10 100 raytracingc_amd/_lib/exact_probe
AB_REPS=3 timeout -k 10 500 bash tools/ab_bench_libs.sh librtc_new.so librtc_nounit.so > gpurun_out/ab_r04_i.log 2>&1 || { echo ab failed; cat gpurun_out/ab_r04_i.log; exit 1; }
cat gpurun_out/ab_r04_i.log
