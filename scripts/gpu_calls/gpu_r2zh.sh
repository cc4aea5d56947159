#!/bin/bash
# fp8 tile kernel with conflict-free fragment reads: fp8 GPU tests, kernel A/B, LDS-conflict PMC, GPT-2-medium fp8/bf16 benches.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_r2h
set -e
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py tests/test_models.py -k "fp8" > gpurun_out/r2zh_tests.log 2>&1
timeout -k 10 300 python scripts/fp8_ab.py > gpurun_out/r2zh_fp8_ab.log 2>&1
timeout -s KILL 150 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE \
   --kernel-trace --output-format csv -d gpurun_out/pmc_r2h -o fp8_a -- python3 scripts/fp8_ab.py > /dev/null 2>&1
python3 scripts/pmc_summary.py $(find gpurun_out/pmc_r2h -name 'fp8*_counter_collection.csv') --match gemm > gpurun_out/pmc_r2h/fp8_summary.txt
find gpurun_out/pmc_r2h -name '*.csv' -size +2M -delete
timeout -k 10 400 python bench.py --model gpt2-medium-fp8 --steps 10 --warmup 3 > gpurun_out/r2zh_bench_fp8.log 2>&1
timeout -k 10 400 python bench.py --model gpt2-medium --steps 10 --warmup 3 > gpurun_out/r2zh_bench_bf16.log 2>&1
