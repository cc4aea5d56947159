#!/bin/bash
# PMC counters per GEMM tile config on single shapes (each rocprofv3 run: --pmc + --kernel-trace only).
#   bash scripts/pmc_gemm_cfg.sh "M N K layout" cfg...      (cfg "torch" = torch.matmul / hipBLASLt)
# Summarise with: python scripts/pmc_summary.py gpurun_out/pmc/*_counter_collection.csv
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
set -e
shape=$1; shift
tag=$(echo "$shape" | tr ' ' '_')
for cfg in "$@"; do
  if [ "$cfg" = torch ]; then sel="--torch"; else sel="--cfg $cfg"; fi
  timeout -k 10 120 python3 scripts/gemm_one.py $shape $sel --iters 20
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
     --kernel-trace --output-format csv -d gpurun_out/pmc -o ${tag}_${cfg}_a -- python3 scripts/gemm_one.py $shape $sel --iters 3 > /dev/null 2>&1
  timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE \
     --kernel-trace --output-format csv -d gpurun_out/pmc -o ${tag}_${cfg}_b -- python3 scripts/gemm_one.py $shape $sel --iters 3 > /dev/null 2>&1
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE \
     --kernel-trace --output-format csv -d gpurun_out/pmc -o ${tag}_${cfg}_c -- python3 scripts/gemm_one.py $shape $sel --iters 3 > /dev/null 2>&1
done
