set -u
export TMPDIR=/tmp
R=$(pwd); mkdir -p gpurun_out
RTC_LIB_PATH=$R/raytracingc_amd/_lib/librtc.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_mc.log 2>&1 || { echo pytest failed; tail -30 gpurun_out/pytest_mc.log; exit 1; }
echo "mc: $(tail -1 gpurun_out/pytest_mc.log)"
for rep in 1 2; do for l in librtc_prev.so librtc.so; do
  RTC_LIB_PATH=$R/raytracingc_amd/_lib/$l timeout -k 10 200 python bench.py --steps 50 --warmup 5 --no-extras --no-cpu-baseline > gpurun_out/b.log 2>&1 || { tail -5 gpurun_out/b.log; exit 1; }
  grep '^{' gpurun_out/b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print('$l', 'static', d['ms_per_step'], 'moving', d['moving_camera']['ms_per_step'])"
done; done
