#!/bin/bash
# GPT-2-medium fp8 vs bf16 50-step loss trajectory (b16 x 1024), lr 1e-4.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
set -e
timeout -k 10 600 python scripts/fp8_trajectory.py 50 16 1e-4 > gpurun_out/r2z_fp8_traj_lr1e-4.jsonl 2> gpurun_out/r2z_fp8_traj.err
