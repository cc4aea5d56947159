#!/bin/bash
# Round-2 status call: benches of every BASELINE config + a GPT-2-small step kernel breakdown.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_r2
set -e
for m in gpt2-small vit-b16 resnet18 gpt2-medium gpt2-medium-fp8; do
  timeout -k 10 400 python bench.py --model $m --steps 10 --warmup 3 > gpurun_out/bench_$m.log 2>&1
  echo "$(tail -1 gpurun_out/bench_$m.log)" >> gpurun_out/bench_all_r2.jsonl
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r2 -o g2s -- python bench.py --steps 5 --warmup 3 --graph off > gpurun_out/prof_r2.log 2>&1
