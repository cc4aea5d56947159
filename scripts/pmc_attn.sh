#!/bin/bash
# PMC counters for the attention kernels (each rocprofv3 run: --pmc + --kernel-trace only).
#   bash scripts/pmc_attn.sh ["<attn_ab.py args>"] [tag]
# Summarise: python scripts/pmc_summary.py gpurun_out/pmc_attn/<tag>*_counter_collection.csv --match attn
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_attn
set -e
ARGS="${1:-64 --rounds 1}"
TAG="${2:-attn}"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE \
   --kernel-trace --output-format csv -d gpurun_out/pmc_attn -o ${TAG}_a -- python3 scripts/attn_ab.py $ARGS > /dev/null 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE SQ_INSTS_MFMA \
   --kernel-trace --output-format csv -d gpurun_out/pmc_attn -o ${TAG}_b -- python3 scripts/attn_ab.py $ARGS > /dev/null 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_VALU_TRANS_F32 GRBM_GUI_ACTIVE \
   --kernel-trace --output-format csv -d gpurun_out/pmc_attn -o ${TAG}_c -- python3 scripts/attn_ab.py $ARGS > /dev/null 2>&1
