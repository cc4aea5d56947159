#!/bin/bash
# PMC counters for single GEMM shapes (each rocprofv3 run: --pmc + --kernel-trace only).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
set -e
i=0
for shape in "16384 768 50304 nn --cfg 6" "16384 2304 768 nt --cfg 6" "16384 768 3072 nt --cfg 6" "50304 768 16384 tn --cfg 1 --split 2"; do
  i=$((i+1))
  timeout -k 10 120 python3 scripts/gemm_one.py $shape --iters 20
  timeout -k 10 120 python3 scripts/gemm_one.py $shape --iters 20 --torch
  timeout -k 10 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
     --kernel-trace --output-format csv -d gpurun_out/pmc -o s${i}a -- python3 scripts/gemm_one.py $shape --iters 5 > /dev/null 2>&1
  timeout -k 10 180 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS \
     --kernel-trace --output-format csv -d gpurun_out/pmc -o s${i}b -- python3 scripts/gemm_one.py $shape --iters 5 > /dev/null 2>&1
done
ls gpurun_out/pmc
