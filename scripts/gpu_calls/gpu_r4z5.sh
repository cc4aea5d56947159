#!/bin/bash
# round 4 (call Z5): PMC counters of the decoding kernels (skinny-M GEMM, one-query attention) in a
# GPT-2-small batch-16 decode run: three rocprofv3 passes (--pmc + --kernel-trace only, per-pass slot
# limits), summarised per kernel template by scripts/pmc_summary.py.
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/pmc_dec; export TMPDIR=/tmp
A="scripts/decode_bench.py --batches 16 --new 16"
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE \
   --kernel-trace --output-format csv -d gpurun_out/pmc_dec -o dec_a -- python3 $A > gpurun_out/pmc_dec_a.log 2>&1 || { echo "pass a failed"; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_MFMA GRBM_GUI_ACTIVE \
   --kernel-trace --output-format csv -d gpurun_out/pmc_dec -o dec_b -- python3 $A > gpurun_out/pmc_dec_b.log 2>&1 || { echo "pass b failed"; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE \
   --kernel-trace --output-format csv -d gpurun_out/pmc_dec -o dec_c -- python3 $A > gpurun_out/pmc_dec_c.log 2>&1 || { echo "pass c failed"; exit 1; }
python scripts/pmc_summary.py gpurun_out/pmc_dec/dec_*_counter_collection.csv > gpurun_out/pmc_dec_summary.txt 2>&1
grep -E "skinny|attn_decode|ln_fwd|index_copy" gpurun_out/pmc_dec_summary.txt | cut -c1-330
exit 0
