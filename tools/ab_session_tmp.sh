set -u
export TMPDIR=/tmp
R=$(pwd); mkdir -p gpurun_out
AB_REPS=3 timeout -k 10 400 bash tools/ab_bench_libs.sh librtc_cur.so librtc_w4.so > gpurun_out/ab_w4.log 2>&1 || { echo ab failed; cat gpurun_out/ab_w4.log; exit 1; }
cat gpurun_out/ab_w4.log
AB_REPS=1 timeout -k 10 300 bash tools/ab_bench_libs.sh --workload fsuzane_1080p64 librtc_cur.so librtc_w4.so > gpurun_out/ab_w4fs.log 2>&1 || { echo ab failed; cat gpurun_out/ab_w4fs.log; exit 1; }
cat gpurun_out/ab_w4fs.log
SCALE_NS=8,4 timeout -k 10 400 bash tools/ab_scale.sh overlap librtc_cur.so librtc_s3.so librtc_cur.so librtc_s3.so > gpurun_out/abs_s3.log 2>&1 || { cat gpurun_out/abs_s3.log; exit 1; }
cat gpurun_out/abs_s3.log
