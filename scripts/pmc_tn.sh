#!/bin/bash
# PMC: wgrad layout (tn) vs fwd layout (nt) at M=3072 N=768 K=65536, cfg1 split 7
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_tn
set -e
for lay in tn nt; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE \
     --kernel-trace --output-format csv -d gpurun_out/pmc_tn -o ${lay}a -- python3 scripts/gemm_one.py 3072 768 65536 $lay --cfg 1 --split 7 --iters 3 > /dev/null 2>&1
  timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU \
     --kernel-trace --output-format csv -d gpurun_out/pmc_tn -o ${lay}b -- python3 scripts/gemm_one.py 3072 768 65536 $lay --cfg 1 --split 7 --iters 3 > /dev/null 2>&1
  timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum \
     --kernel-trace --output-format csv -d gpurun_out/pmc_tn -o ${lay}c -- python3 scripts/gemm_one.py 3072 768 65536 $lay --cfg 1 --split 7 --iters 3 > /dev/null 2>&1 || true
done
ls gpurun_out/pmc_tn
