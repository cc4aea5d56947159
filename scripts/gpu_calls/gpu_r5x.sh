#!/bin/bash
# round 5 (call X): early-descent fp8 deviation vs delayed-scaling headroom, with the fp8 head and fp8 attention c_proj
# (the new defaults): 50-step trajectories (+ held-out eval) at headroom 2 (default), 4, 8 and gradient headroom 4.
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
t() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 400 python -u scripts/fp8_trajectory.py 50 16 1e-4 > gpurun_out/r5x_traj_$tag.jsonl 2> gpurun_out/r5x_traj_$tag.err || { echo "trajectory $tag failed"; tail -5 gpurun_out/r5x_traj_$tag.err; exit 1; }
  echo "$tag: $(grep summary gpurun_out/r5x_traj_$tag.jsonl)"
}
t hr2 REPLICANN_X=0 || exit 1
t hr4 REPLICANN_FP8_HEADROOM=4 REPLICANN_FP8_GHEADROOM=4 || exit 1
t hr8 REPLICANN_FP8_HEADROOM=8 REPLICANN_FP8_GHEADROOM=8 || exit 1
t ghr4 REPLICANN_FP8_GHEADROOM=4 || exit 1
