#!/bin/bash
# PMC of the one-wave-per-SIMD GEMM (cfg 11) against cfg 9 on single shapes: 2 counter passes per run
# (--pmc + --kernel-trace only), 60-s kill limits.   bash scripts/pmc_w1.sh OUTDIR "M N K layout [extra args]"...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=$1; shift
mkdir -p "$out"
set -e
i=0
for spec in "$@"; do
  i=$((i + 1))
  timeout -k 10 120 python3 scripts/gemm_one.py $spec --iters 20
  timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE \
     --kernel-trace --output-format csv -d "$out" -o run${i}_a -- python3 scripts/gemm_one.py $spec --iters 3 > /dev/null 2>&1
  timeout -s KILL 60 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE \
     --kernel-trace --output-format csv -d "$out" -o run${i}_b -- python3 scripts/gemm_one.py $spec --iters 3 > /dev/null 2>&1
done
