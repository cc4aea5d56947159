#!/bin/bash
# Round-2 PMC passes: attention D=64 fwd/bwd (B64 H12 T1024 causal), CE row kernel v2 (+ v1), fp8 GEMMs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_r2
set -e
bash scripts/pmc_attn.sh "64 --fwd 3 --bwd 1 --rounds 1" r2attn
P=gpurun_out/pmc_r2
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 GRBM_GUI_ACTIVE \
   --kernel-trace --output-format csv -d $P -o xent_a -- python3 scripts/xent_ab.py > /dev/null 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $P -o xent_b -- python3 scripts/xent_ab.py > /dev/null 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $P -o xent_c -- python3 scripts/xent_ab.py > /dev/null 2>&1
timeout -s KILL 150 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE \
   --kernel-trace --output-format csv -d $P -o fp8_a -- python3 scripts/fp8_ab.py > /dev/null 2>&1
python3 scripts/pmc_summary.py $(find gpurun_out/pmc_attn -name 'r2attn*_counter_collection.csv') --match attn > $P/attn_summary.txt
python3 scripts/pmc_summary.py $(find $P -name 'xent*_counter_collection.csv') --match xent > $P/xent_summary.txt
python3 scripts/pmc_summary.py $(find $P -name 'fp8*_counter_collection.csv') --match gemm > $P/fp8_summary.txt
find gpurun_out/pmc_attn $P -name '*.csv' -size +2M -delete
