#!/bin/bash
# Quick PMC passes (each its own run and time limit) over one faithful 1080p x64 render; summaries per kernel.
# usage: tools/pmc_quick.sh <tag> [one_render variant]
set -u
export TMPDIR=/tmp
R=$(pwd); OUT=$R/gpurun_out; tag=$1; v=${2:-faithful}
mkdir -p "$OUT"; cd /tmp
run() { local name=$1; shift; timeout -s KILL 90 rocprofv3 --kernel-trace --pmc "$@" -d "$OUT/pmc_$tag/$name" -o p --output-format csv -- python3 "$R/tools/one_render.py" $v 2 > "$OUT/pmc_${tag}_$name.log" 2>&1 || { echo "pass $name failed"; exit 1; }; }
run a SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE
run b SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT
run c SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR
cd "$R" && python3 tools/pmc_summary.py "$OUT/pmc_$tag" > "$OUT/pmc_${tag}_summary.txt" 2>&1; cat "$OUT/pmc_${tag}_summary.txt"
