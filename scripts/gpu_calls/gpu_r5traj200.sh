#!/bin/bash
# round 5: a 200-step GPT-2-medium fp8 (final defaults) vs bf16 trajectory with the held-out eval loss
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u scripts/fp8_trajectory.py 200 16 1e-4 > gpurun_out/r5t200_traj.jsonl 2> gpurun_out/r5t200_traj.err || { echo "trajectory failed"; tail -5 gpurun_out/r5t200_traj.err; exit 1; }
grep summary gpurun_out/r5t200_traj.jsonl
