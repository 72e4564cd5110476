set -u
export TMPDIR=/tmp
R=$(pwd); mkdir -p gpurun_out
for v in cs5; do
RTC_LIB_PATH=$R/raytracingc_amd/_lib/librtc_$v.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_$v.log 2>&1 || { echo pytest $v failed; tail -30 gpurun_out/pytest_$v.log; exit 1; }
echo "$v: $(tail -1 gpurun_out/pytest_$v.log)"
done
SCALE_NS=2 timeout -k 10 400 bash tools/ab_scale.sh overlap librtc_cur.so librtc_cs4.so librtc_cs5.so librtc_cur.so librtc_cs4.so librtc_cs5.so > gpurun_out/abs_cs5.log 2>&1 || { cat gpurun_out/abs_cs5.log; exit 1; }
cat gpurun_out/abs_cs5.log
for l in librtc_cur.so librtc_cs4.so librtc_cs5.so; do
  RTC_LIB_PATH=$R/raytracingc_amd/_lib/$l SCALE_NS=8,4 timeout -k 10 240 python tools/scale_probe.py 5 3840 2160 64 overlap > gpurun_out/abs4k.log 2>&1 || { tail -5 gpurun_out/abs4k.log; exit 1; }
  sed "s/^/$l 4k /" gpurun_out/abs4k.log | grep '"n"'
done
