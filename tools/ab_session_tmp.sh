set -u
export TMPDIR=/tmp
R=$(pwd); mkdir -p gpurun_out
AB_REPS=3 timeout -k 10 500 bash tools/ab_bench_libs.sh librtc_new.so librtc_nofb.so librtc_fbcall.so librtc_fbser.so > gpurun_out/ab_r04_o.log 2>&1 || { echo ab failed; cat gpurun_out/ab_r04_o.log; exit 1; }
cat gpurun_out/ab_r04_o.log
SCALE_NS=8 timeout -k 10 400 bash tools/ab_scale.sh overlap librtc_new.so librtc_fbcall.so librtc_fbser.so librtc_new.so librtc_fbcall.so librtc_fbser.so > gpurun_out/abs_r04_o.log 2>&1 || { cat gpurun_out/abs_r04_o.log; exit 1; }
cat gpurun_out/abs_r04_o.log
