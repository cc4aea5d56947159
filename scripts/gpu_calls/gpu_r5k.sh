#!/bin/bash
# round 5 (call K): the all-fp8 MLP keeping h (gelu_q8 pass, gelu'(h) re-derived in the fused backward):
# tests, GPT-2-medium bf16 / fp8 / fp8 + fp8 c_proj alternating, breakdown, trajectories (fp8, fp8 + c_proj).
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
PT="python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 400 $PT tests/test_fp8_wgrad_gpu.py tests/test_fp8_inference_gpu.py tests/test_ops_gpu.py -k "fp8 or mlp or gelu or act_mul" > gpurun_out/r5k_tests.log 2>&1; rc=$?
echo "=== tests rc=$rc"; grep -E "FAILED|passed|failed" gpurun_out/r5k_tests.log | tail -8
[ $rc -eq 0 ] || exit $rc
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 240 python -u bench.py --model ${M} --steps 6 --warmup 3 > gpurun_out/r5k_$tag.log 2>&1 || { echo "bench $tag failed"; tail -5 gpurun_out/r5k_$tag.log; exit 1; }
  echo "$tag: $(grep -o '"value": [0-9.]*' gpurun_out/r5k_$tag.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5k_$tag.log) $(grep -o '"loss_first_last": [^]]*]' gpurun_out/r5k_$tag.log)"
}
for r in 1 2; do
  M=gpt2-medium run bf16_$r REPLICANN_X=0 || exit 1
  M=gpt2-medium-fp8 run fp8_$r REPLICANN_X=0 || exit 1
  M=gpt2-medium-fp8 run fp8proj_$r REPLICANN_FP8_PROJ=1 || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_5k -o run -- python3 bench.py --model gpt2-medium-fp8 --steps 3 --warmup 2 > gpurun_out/r5k_prof.log 2>&1 || { echo "prof failed"; exit 1; }
python scripts/prof_steps.py gpurun_out/prof_5k/run_kernel_trace.csv --steps 3 > gpurun_out/r5k_steps_m8.txt 2>&1
rm -rf gpurun_out/prof_5k
head -24 gpurun_out/r5k_steps_m8.txt | cut -c1-150
timeout -k 10 500 python -u scripts/fp8_trajectory.py 50 16 1e-4 > gpurun_out/r5k_traj.jsonl 2> gpurun_out/r5k_traj.err || { echo "trajectory failed"; tail -5 gpurun_out/r5k_traj.err; exit 1; }
grep summary gpurun_out/r5k_traj.jsonl
REPLICANN_FP8_PROJ=1 timeout -k 10 500 python -u scripts/fp8_trajectory.py 50 16 1e-4 > gpurun_out/r5k_traj_proj.jsonl 2> gpurun_out/r5k_traj_proj.err || { echo "trajectory proj failed"; tail -5 gpurun_out/r5k_traj_proj.err; exit 1; }
grep summary gpurun_out/r5k_traj_proj.jsonl
