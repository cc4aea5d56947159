#!/bin/bash
# Round-2 GPU call: parity vs recorded reference outputs, then GEMM PMC record (cfg 9 vs hipBLASLt).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
set -e
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_reference_parity_gpu.py -m gpu > gpurun_out/parity.log 2>&1
for s in "65536 2304 768 nt" "65536 768 3072 nt" "65536 50304 768 nt" "65536 768 50304 nn" "2304 768 65536 tn"; do
  bash scripts/pmc_gemm_cfg.sh "$s" 9 torch >> gpurun_out/pmc_times.log 2>&1
done
python scripts/pmc_summary.py gpurun_out/pmc/*_counter_collection.csv --match "" > gpurun_out/pmc_summary.txt
