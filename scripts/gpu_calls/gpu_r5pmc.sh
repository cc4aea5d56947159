#!/bin/bash
# round 5: PMC of the halo-tile 3x3 conv (conv3x3.hip) vs the implicit GEMM on ResNet layer 1 (scripts/conv3_one.py):
# two counter passes each (--pmc + --kernel-trace only), 60-s kill limits.
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/pmc_conv3; export TMPDIR=/tmp
set -e
for v in 1 0; do
  timeout -k 10 120 env REPLICANN_CONV3X3=$v python3 scripts/conv3_one.py 3
  REPLICANN_CONV3X3=$v timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE \
     --kernel-trace --output-format csv -d gpurun_out/pmc_conv3 -o c3_${v}_a -- python3 scripts/conv3_one.py 3 > /dev/null 2>&1
  REPLICANN_CONV3X3=$v timeout -s KILL 60 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA GRBM_GUI_ACTIVE \
     --kernel-trace --output-format csv -d gpurun_out/pmc_conv3 -o c3_${v}_b -- python3 scripts/conv3_one.py 3 > /dev/null 2>&1
done
python3 scripts/pmc_summary.py gpurun_out/pmc_conv3/*_counter_collection.csv > gpurun_out/pmc_conv3_summary.txt 2>&1 || true
find gpurun_out/pmc_conv3 -name "*.csv" | head -3
cut -c1-260 gpurun_out/pmc_conv3_summary.txt | grep -E "conv3x3|gemm_k|run|c3" | head -20
