#!/bin/bash
# Round-2 GPU call: stochastic-rounding test, trajectory with SR (b16, b64) and without (b16).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
set -e
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_ops_gpu.py -k "adamw or optim" tests/test_determinism_gpu.py > gpurun_out/sr_tests.log 2>&1
timeout -k 10 400 python -u scripts/check_trajectory.py --model gpt2-small --batch 16 --steps 100 --lr 1e-4 --warmup 10 --threshold 0.02 > gpurun_out/traj_sr16.jsonl 2> gpurun_out/traj.err || true
timeout -k 10 600 python -u scripts/check_trajectory.py --model gpt2-small --batch 64 --steps 100 --lr 1e-4 --warmup 10 --threshold 0.02 > gpurun_out/traj_sr64.jsonl 2>> gpurun_out/traj.err || true
