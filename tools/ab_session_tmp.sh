set -u
export TMPDIR=/tmp
R=$(pwd); mkdir -p gpurun_out
AB_REPS=2 timeout -k 10 500 bash tools/ab_bench_libs.sh librtc_new.so librtc_c768.so librtc_c512.so librtc_c768inl.so librtc_inl.so > gpurun_out/ab_r04_g.log 2>&1 || { echo ab failed; cat gpurun_out/ab_r04_g.log; exit 1; }
cat gpurun_out/ab_r04_g.log
cd /tmp
for v in c768 c512 c768inl; do
RTC_LIB_PATH=$R/raytracingc_amd/_lib/librtc_$v.so timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/loop1_${v}_r04_g -o run --output-format csv -- python3 $R/tools/frame_loop.py 40 overlap 1 > $R/gpurun_out/loop1_${v}_r04_g.log 2>&1 || exit 1
echo "== $v"; python3 $R/tools/trace_timeline.py $R/gpurun_out/loop1_${v}_r04_g/run_kernel_trace.csv 2
done
