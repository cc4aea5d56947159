#!/bin/bash
# round 5 (call G): GPT-2-medium bf16 vs fp8 with the one-wave-per-SIMD fp8 kernels now also behind the data
# and weight gradients (REPLICANN_FP8_DGRAD / _WGRAD), alternating; 50-step fp8 (fwd + dgrad + wgrad) vs bf16
# loss trajectory.
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
run() {  # tag, env..., model
  local tag=$1; shift
  env "$@" timeout -k 10 240 python -u bench.py --model ${M} --steps 6 --warmup 3 > gpurun_out/r5g_$tag.log 2>&1 || { echo "bench $tag failed"; tail -5 gpurun_out/r5g_$tag.log; exit 1; }
  echo "$tag: $(grep -o '"value": [0-9.]*' gpurun_out/r5g_$tag.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5g_$tag.log)"
}
for r in 1 2; do
  M=gpt2-medium run bf16_$r REPLICANN_X=0 || exit 1
  M=gpt2-medium-fp8 run fp8fwd_$r REPLICANN_X=0 || exit 1
  M=gpt2-medium-fp8 run fp8dgrad_$r REPLICANN_FP8_DGRAD=1 || exit 1
  M=gpt2-medium-fp8 run fp8all_$r REPLICANN_FP8_DGRAD=1 REPLICANN_FP8_WGRAD=1 || exit 1
done
REPLICANN_FP8_DGRAD=1 REPLICANN_FP8_WGRAD=1 timeout -k 10 500 python -u scripts/fp8_trajectory.py 50 16 1e-4 > gpurun_out/r5g_traj.jsonl 2> gpurun_out/r5g_traj.err || { echo "trajectory failed"; tail -5 gpurun_out/r5g_traj.err; exit 1; }
grep summary gpurun_out/r5g_traj.jsonl
