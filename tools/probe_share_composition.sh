set -u
export TMPDIR=/tmp
OUT=gpurun_out/probe_d.log; : > $OUT
run() { echo "== $*" >> $OUT; timeout -k 10 150 "$@" 2>/dev/null | grep '^{' >> $OUT || { echo FAIL >> $OUT; exit 1; }; }
export SCALE_NS=1,8
run python tools/scale_probe.py 5 1920 1080 64 overlap
run python tools/scale_probe.py 5 1920 1080 64 overlap_hoist
run python tools/scale_probe.py 5 1920 1080 32 overlap
run python tools/scale_probe.py 5 1920 1080 16 overlap
run python tools/scale_probe.py 5 1920 1080 1 overlap
RTC_LIB_PATH=$PWD/raytracingc_amd/_lib/librtc_cheapsky.so run python tools/scale_probe.py 5 1920 1080 64 overlap
cat $OUT
