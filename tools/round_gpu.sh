#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, variant probe, rocprofv3 kernel-trace summary and the PMC
# passes (one counter group per run).  Every GPU step has its own time limit; the script stops at the first
# failing step.  usage: tools/round_gpu.sh [all|tests|bench|prof]
set -u
export TMPDIR=/tmp
R=$(pwd)
OUT=$R/gpurun_out
mkdir -p "$OUT"
what=${1:-all}
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "== $name $(date +%T)" | tee -a "$OUT/steps.log"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc" | tee -a "$OUT/steps.log"
  tail -4 "$OUT/$name.log"
  return $rc
}
if [ "$what" = all ] || [ "$what" = tests ]; then
  step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v -s --timeout 120 --timeout-method thread -p no:cacheprovider || exit $?
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
fi
if [ "$what" = all ] || [ "$what" = bench ]; then
  step bench 600 python bench.py --steps 10 --warmup 2 || exit $?
  step probe 300 python tools/kernel_probe.py --quick || exit $?
fi
if [ "$what" = all ] || [ "$what" = prof ]; then
  cd /tmp
  step rocprof 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu-baseline --no-hoisted || exit $?
  step pmc_fetch 90 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o p --output-format csv -- python3 "$R/tools/one_render.py" faithful 2 || exit $?
  step pmc_write 90 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d "$OUT/pmc_write" -o p --output-format csv -- python3 "$R/tools/one_render.py" faithful 2 || exit $?
  cd "$R" && python3 tools/pmc_traffic.py "$OUT" > "$OUT/pmc_traffic.log" 2>&1; cd /tmp
  step pmc_sq 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE -d "$OUT/pmc_sq" -o p --output-format csv -- python3 "$R/tools/one_render.py" faithful 2 || exit $?
fi
echo done
