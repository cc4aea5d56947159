#!/bin/bash
# round 5 (call P): the fp8 LM head modes 1 / 2 vs 0 (bench + trajectories with a held-out eval loss); (REPLICANN_FP8_HEAD=1: e4m3 logits GEMM, e5m2 loss gradient from the CE
# kernel, fp8 head gradients).  Tests, GPT-2-medium fp8 with / without it alternating, breakdown, trajectory.
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
PT="python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 500 $PT tests/test_fp8_head_gpu.py > gpurun_out/r5p_tests.log 2>&1; rc=$?
echo "=== tests rc=$rc"; grep -E "FAILED|Error|passed|failed" gpurun_out/r5p_tests.log | tail -6
[ $rc -eq 0 ] || exit $rc
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 240 python -u bench.py --model ${M} --steps 6 --warmup 3 > gpurun_out/r5p_$tag.log 2>&1 || { echo "bench $tag failed"; tail -5 gpurun_out/r5p_$tag.log; exit 1; }
  echo "$tag: $(grep -o '"value": [0-9.]*' gpurun_out/r5p_$tag.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5p_$tag.log)"
}
for r in 1 2; do
  M=gpt2-medium run bf16_$r REPLICANN_X=0 || exit 1
  M=gpt2-medium-fp8 run fp8_$r REPLICANN_X=0 || exit 1
  M=gpt2-medium-fp8 run head1_$r REPLICANN_FP8_HEAD=1 || exit 1
  M=gpt2-medium-fp8 run head2_$r REPLICANN_FP8_HEAD=2 || exit 1
done
t() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 400 python -u scripts/fp8_trajectory.py 50 16 1e-4 > gpurun_out/r5p_traj_$tag.jsonl 2> gpurun_out/r5p_traj_$tag.err || { echo "trajectory $tag failed"; tail -5 gpurun_out/r5p_traj_$tag.err; exit 1; }
  echo "$tag: $(grep summary gpurun_out/r5p_traj_$tag.jsonl)"
}
t head0 REPLICANN_FP8_HEAD=0 || exit 1
t head1 REPLICANN_FP8_HEAD=1 || exit 1
t head2 REPLICANN_FP8_HEAD=2 || exit 1
