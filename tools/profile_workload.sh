#!/bin/bash
# rocprofv3 evidence of one workload (run on the GPU box): a kernel trace of the bench command and PMC passes, one
# counter group per run, each under its own time limit, over tools/one_render.py <workload>; outputs under
# gpurun_out/prof_<workload>_<tag>/ (digest: tools/pmc_digest.py).  usage: tools/profile_workload.sh <workload> <tag>
set -u
export TMPDIR=/tmp
R=$(pwd)
w=${1:-ultracomplex_1080p64}; tag=${2:-r03}
OUT=$R/gpurun_out/prof_${w}_${tag}
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
step trace 240 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 "$R/bench.py" --workload "$w" --steps 20 --warmup 3 --no-cpu-baseline --no-extras || exit $?
G1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY"
G2="SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_INT32"
G3="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_BRANCH GRBM_GUI_ACTIVE"
g=0
for grp in "$G1" "$G2" "$G3" "FETCH_SIZE" "WRITE_SIZE"; do
  g=$((g + 1))
  step pmc_g$g 90 rocprofv3 --kernel-trace --pmc $grp -d "$OUT/pmc_g$g" -o p --output-format csv -- python3 "$R/tools/one_render.py" "$w" 2 || exit $?
done
echo done
