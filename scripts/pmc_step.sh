#!/bin/bash
# PMC counters for every kernel of a training step (each rocprofv3 run: --pmc + --kernel-trace only,
# counter sets within the per-pass slot limits: 8 SQ, 4 TCC, 2 GRBM).
#   bash scripts/pmc_step.sh ["<bench.py args>"] [tag]
# Summarise: python scripts/pmc_summary.py gpurun_out/pmc_step/<tag>*_counter_collection.csv
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_step
set -e
ARGS="${1:---steps 2 --warmup 1}"
TAG="${2:-step}"
export REPLICANN_GEMM_AUTOTUNE=0  # the committed tuning tables only: no candidate-timing dispatches
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE \
   --kernel-trace --output-format csv -d gpurun_out/pmc_step -o ${TAG}_a -- python3 bench.py $ARGS > /dev/null 2>&1
timeout -s KILL 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_MFMA GRBM_GUI_ACTIVE \
   --kernel-trace --output-format csv -d gpurun_out/pmc_step -o ${TAG}_b -- python3 bench.py $ARGS > /dev/null 2>&1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE \
   --kernel-trace --output-format csv -d gpurun_out/pmc_step -o ${TAG}_c -- python3 bench.py $ARGS > /dev/null 2>&1
