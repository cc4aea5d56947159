#!/bin/bash
# round 5 (call N): fp8 accuracy A/B — 50-step GPT-2-medium trajectories vs bf16: default (headroom 2), headroom 1
# (REPLICANN_FP8_HEADROOM=1 / GHEADROOM=1), forward-only fp8 (REPLICANN_FP8_WGRAD=0 / DGRAD=0).
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
t() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 400 python -u scripts/fp8_trajectory.py 50 16 1e-4 > gpurun_out/r5n_traj_$tag.jsonl 2> gpurun_out/r5n_traj_$tag.err || { echo "trajectory $tag failed"; tail -5 gpurun_out/r5n_traj_$tag.err; exit 1; }
  echo "$tag: $(grep summary gpurun_out/r5n_traj_$tag.jsonl)"
}
t default REPLICANN_X=0 || exit 1
t hr1 REPLICANN_FP8_HEADROOM=1 REPLICANN_FP8_GHEADROOM=1 || exit 1
t ghr1 REPLICANN_FP8_GHEADROOM=1 || exit 1
t fwdonly REPLICANN_FP8_WGRAD=0 REPLICANN_FP8_DGRAD=0 || exit 1
