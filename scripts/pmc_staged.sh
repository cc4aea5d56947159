#!/bin/bash
# PMC counters of the persistent GEMM's full-tile-operand epilogues, staged (default) vs unstaged
# (REPLICANN_GEMM_STAGED=0): attention c_proj forward + residual, MLP c_proj forward + residual, fc1
# dgrad with the saved gelu' (code 6).  Each rocprofv3 run: --pmc + --kernel-trace only.
#   bash scripts/pmc_staged.sh;  python scripts/pmc_summary.py gpurun_out/pmc_stg/*_counter_collection.csv --match gemm_pk
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_stg
set -e
i=0
for shape in "65536 768 768 nt --res --bias" "65536 768 3072 nt --res --bias" "65536 3072 768 nn --act 6"; do
  i=$((i+1))
  for stg in 1 0; do
    export REPLICANN_GEMM_STAGED=$stg
    timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE \
       --kernel-trace --output-format csv -d gpurun_out/pmc_stg -o s${i}_stg${stg}_a -- python3 scripts/gemm_one.py $shape --cfg 9 --split 1 --iters 5 > /dev/null 2>&1
    timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE \
       --kernel-trace --output-format csv -d gpurun_out/pmc_stg -o s${i}_stg${stg}_b -- python3 scripts/gemm_one.py $shape --cfg 9 --split 1 --iters 5 > /dev/null 2>&1
  done
done
unset REPLICANN_GEMM_STAGED
