#!/bin/bash
# rocprofv3 evidence for profiles/: kernel-trace stats of a short bench run, and PMC passes (one counter group
# per run, each under its own time limit) over one faithful 1080p x64 render.  usage: tools/prof_session.sh [tag]
set -u
export TMPDIR=/tmp
R=$(pwd)
OUT=$R/gpurun_out
tag=${1:-r02}
mkdir -p "$OUT"
cd /tmp
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "== $name $(date +%T)" | tee -a "$OUT/steps.log"
  timeout -s KILL "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc" | tee -a "$OUT/steps.log"
  return $rc
}
step "list_$tag" 60 rocprofv3 -L || true
step "trace_$tag" 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace_$tag" -o run --output-format csv -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu-baseline --no-extras || exit $?
step "pmc_sq_$tag" 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE -d "$OUT/pmc_sq_$tag" -o p --output-format csv -- python3 "$R/tools/one_render.py" faithful 2 || exit $?
step "pmc_fetch_$tag" 90 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o p --output-format csv -- python3 "$R/tools/one_render.py" faithful 2 || exit $?
step "pmc_write_$tag" 90 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d "$OUT/pmc_write" -o p --output-format csv -- python3 "$R/tools/one_render.py" faithful 2 || exit $?
echo done
