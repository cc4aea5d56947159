#!/bin/bash
# Round-2 per-step kernel breakdowns: ViT-B/16 b512 and ResNet-18 b256 (eager), plus their graph benches.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_r2x
set -e
timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/prof_r2x/vit -o vit -- python bench.py --model vit-b16 --steps 5 --warmup 3 --graph off > gpurun_out/prof_r2x/vit.log 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/prof_r2x/rn -o rn -- python bench.py --model resnet18 --steps 5 --warmup 3 --graph off > gpurun_out/prof_r2x/rn.log 2>&1
python scripts/prof_steps.py "$(find gpurun_out/prof_r2x/vit -name '*.db' | head -n1)" --steps 5 --per-step 12 --top 30 > gpurun_out/prof_r2x/vit_steps.txt
python scripts/prof_steps.py "$(find gpurun_out/prof_r2x/rn -name '*.db' | head -n1)" --steps 5 --per-step 1 --marker sgd_k --top 30 > gpurun_out/prof_r2x/rn_steps.txt || true
find gpurun_out/prof_r2x -name "*.db" -delete
timeout -k 10 300 python bench.py --model vit-b16 --steps 10 --warmup 3 > gpurun_out/prof_r2x/vit_bench.log 2>&1
timeout -k 10 300 python bench.py --model resnet18 --steps 20 --warmup 3 > gpurun_out/prof_r2x/rn_bench.log 2>&1
