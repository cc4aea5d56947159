#!/bin/bash
# round 5 (call V): the attention c_proj in fp8 too (REPLICANN_FP8_PROJ=1) on top of the fp8 head: bench alternating
# with the default fp8 model, and a 50-step trajectory with the held-out eval loss.
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 240 python -u bench.py --model gpt2-medium-fp8 --steps 6 --warmup 3 > gpurun_out/r5v_$tag.log 2>&1 || { echo "bench $tag failed"; tail -5 gpurun_out/r5v_$tag.log; exit 1; }
  echo "$tag: $(grep -o '"value": [0-9.]*' gpurun_out/r5v_$tag.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5v_$tag.log)"
}
for r in 1 2; do
  run fp8_$r REPLICANN_X=0 || exit 1
  run proj_$r REPLICANN_FP8_PROJ=1 || exit 1
done
REPLICANN_FP8_PROJ=1 timeout -k 10 400 python -u scripts/fp8_trajectory.py 50 16 1e-4 > gpurun_out/r5v_traj_proj.jsonl 2> gpurun_out/r5v_traj_proj.err || { echo "trajectory failed"; tail -5 gpurun_out/r5v_traj_proj.err; exit 1; }
echo "traj proj: $(grep summary gpurun_out/r5v_traj_proj.jsonl)"
