set -u
export TMPDIR=/tmp
R=$(pwd); mkdir -p gpurun_out
for v in altf; do
RTC_LIB_PATH=$R/raytracingc_amd/_lib/librtc_$v.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_$v.log 2>&1 || { echo pytest $v failed; tail -30 gpurun_out/pytest_$v.log; exit 1; }
echo "$v: $(tail -1 gpurun_out/pytest_$v.log)"
done
AB_REPS=3 timeout -k 10 400 bash tools/ab_bench_libs.sh librtc_new.so librtc_altf.so > gpurun_out/ab_altf.log 2>&1 || { echo ab failed; cat gpurun_out/ab_altf.log; exit 1; }
cat gpurun_out/ab_altf.log
AB_REPS=1 timeout -k 10 400 bash tools/ab_bench_libs.sh --workload ultracomplex_4k64 librtc_new.so librtc_altf.so > gpurun_out/ab_altf4k.log 2>&1 || { echo ab failed; cat gpurun_out/ab_altf4k.log; exit 1; }
cat gpurun_out/ab_altf4k.log
cd /tmp
v=altf
RTC_LIB_PATH=$R/raytracingc_amd/_lib/librtc_$v.so timeout -k 10 120 rocprofv3 --kernel-trace -d "$R/gpurun_out/loop_$v" -o run --output-format csv -- python3 "$R/tools/frame_loop.py" 40 overlap 1 > "$R/gpurun_out/loop_$v.log" 2>&1 || { tail -5 "$R/gpurun_out/loop_$v.log"; exit 1; }
echo "== $v"; python3 "$R/tools/trace_timeline.py" $(find "$R/gpurun_out/loop_$v" -name "*kernel_trace.csv") 3
