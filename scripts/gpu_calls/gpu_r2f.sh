#!/bin/bash
# Round-2 GPU call: GPT-2-medium bf16 vs fp8 benches + kernel stats of the fp8 step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_fp8
set -e
timeout -k 10 300 python bench.py --model gpt2-medium --steps 10 --warmup 3 > gpurun_out/bench_med.log 2>&1
timeout -k 10 300 python bench.py --model gpt2-medium-fp8 --steps 10 --warmup 3 > gpurun_out/bench_med_fp8.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fp8 -o fp8 -- python bench.py --model gpt2-medium-fp8 --steps 5 --warmup 3 --graph off > gpurun_out/prof_fp8.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fp8 -o bf16 -- python bench.py --model gpt2-medium --steps 5 --warmup 3 --graph off > gpurun_out/prof_bf16.log 2>&1
