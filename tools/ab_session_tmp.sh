set -u
export TMPDIR=/tmp
R=$(pwd); mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r04_k.log 2>&1 || { echo tests failed; tail -30 gpurun_out/pytest_r04_k.log; exit 1; }
tail -2 gpurun_out/pytest_r04_k.log
AB_REPS=2 timeout -k 10 500 bash tools/ab_bench_libs.sh librtc_new.so librtc_nocst.so > gpurun_out/ab_r04_k.log 2>&1 || { echo ab failed; cat gpurun_out/ab_r04_k.log; exit 1; }
cat gpurun_out/ab_r04_k.log
SCALE_NS=1,8 timeout -k 10 400 bash tools/ab_scale.sh overlap librtc_new.so librtc_nocst.so librtc_new.so librtc_nocst.so > gpurun_out/abs_r04_k.log 2>&1 || { cat gpurun_out/abs_r04_k.log; exit 1; }
cat gpurun_out/abs_r04_k.log
cd /tmp
for v in new nocst; do
RTC_LIB_PATH=$R/raytracingc_amd/_lib/librtc_$v.so timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/loop8_${v}_r04_k -o run --output-format csv -- python3 $R/tools/frame_loop.py 60 overlap 8 > /dev/null 2>&1 || exit 1
echo "== $v share"; python3 $R/tools/trace_timeline.py $R/gpurun_out/loop8_${v}_r04_k/run_kernel_trace.csv 2
RTC_LIB_PATH=$R/raytracingc_amd/_lib/librtc_$v.so timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/loop1_${v}_r04_k -o run --output-format csv -- python3 $R/tools/frame_loop.py 40 overlap 1 > /dev/null 2>&1 || exit 1
echo "== $v full"; python3 $R/tools/trace_timeline.py $R/gpurun_out/loop1_${v}_r04_k/run_kernel_trace.csv 2
done
