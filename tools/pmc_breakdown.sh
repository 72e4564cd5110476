#!/bin/bash
# Instruction-mix / stall breakdown of the render kernel for a few variants (tools/one_render.py), one
# rocprofv3 counter group per run.  usage: tools/pmc_breakdown.sh variant...
set -u
export TMPDIR=/tmp
R=$(pwd)
OUT=$R/gpurun_out/pmcb
mkdir -p "$OUT"
G1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
G2="SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_INT32"
G3="SQ_WAIT_ANY SQ_INST_CYCLES_VMEM_RD SQ_INSTS_BRANCH SQ_INSTS_VALU_CVT SQ_INSTS_VALU_TRANS_F32 SQ_THREAD_CYCLES_VALU SQ_INST_CYCLES_SALU SQ_INST_CYCLES_SMEM"
G4="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAVES"
cd /tmp
for v in "$@"; do
  g=0
  for grp in "$G1" "$G2" "$G3" "$G4"; do
    g=$((g + 1))
    timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $grp -d "$OUT/${v}_g$g" -o p --output-format csv -- python3 "$R/tools/one_render.py" "$v" 1 > "$OUT/${v}_g$g.log" 2>&1
    rc=$?
    echo "$v g$g rc=$rc"
    [ $rc -eq 0 ] || exit $rc
  done
done
