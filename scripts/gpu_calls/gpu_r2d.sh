#!/bin/bash
# Round-2 GPU call: full GPU test suite, GPT-2-small native-vs-fp32 100-step trajectory, N=1 bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
set -e
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/gpu_all.log 2>&1
timeout -k 10 600 python -u scripts/check_trajectory.py --model gpt2-small --steps 100 --lr 1e-4 --warmup 10 \
  --threshold 0.02 > gpurun_out/traj.jsonl 2> gpurun_out/traj.err
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1
