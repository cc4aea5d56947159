#!/bin/bash
# Per-kernel step breakdown of GPT-2-medium fp8 (LayerNorm- and epilogue-fed e4m3) and bf16, eager.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_r2w
set -e
timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/prof_r2w/fp8 -o med_fp8 -- python bench.py --model gpt2-medium-fp8 --steps 5 --warmup 3 --graph off > gpurun_out/prof_r2w/fp8.log 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/prof_r2w/bf16 -o med_bf16 -- python bench.py --model gpt2-medium --steps 5 --warmup 3 --graph off > gpurun_out/prof_r2w/bf16.log 2>&1
find gpurun_out/prof_r2w -name "*.db" > gpurun_out/prof_r2w/dbs.txt
python scripts/prof_steps.py "$(find gpurun_out/prof_r2w/fp8 -name '*.db' | head -n1)" --steps 5 --per-step 24 --top 30 > gpurun_out/prof_r2w/fp8_steps.txt
python scripts/prof_steps.py "$(find gpurun_out/prof_r2w/bf16 -name '*.db' | head -n1)" --steps 5 --per-step 24 --top 30 > gpurun_out/prof_r2w/bf16_steps.txt
find gpurun_out/prof_r2w -name "*.db" -delete
