#!/bin/bash
# round 5 (call O): the fp8 LM head (REPLICANN_FP8_HEAD=1: e4m3 logits GEMM, e5m2 loss gradient from the CE
# kernel, fp8 head gradients).  Tests, GPT-2-medium fp8 with / without it alternating, breakdown, trajectory.
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
PT="python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 500 $PT tests/test_fp8_head_gpu.py tests/test_fp8_wgrad_gpu.py tests/test_gemm_w1_gpu.py tests/test_fp8_inference_gpu.py > gpurun_out/r5o_tests.log 2>&1; rc=$?
echo "=== tests rc=$rc"; grep -E "FAILED|Error|passed|failed" gpurun_out/r5o_tests.log | tail -6
[ $rc -eq 0 ] || exit $rc
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 240 python -u bench.py --model ${M} --steps 6 --warmup 3 > gpurun_out/r5o_$tag.log 2>&1 || { echo "bench $tag failed"; tail -5 gpurun_out/r5o_$tag.log; exit 1; }
  echo "$tag: $(grep -o '"value": [0-9.]*' gpurun_out/r5o_$tag.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5o_$tag.log)"
}
M=gpt2-medium run bf16_1 REPLICANN_X=0 || exit 1
for r in 1 2; do
  M=gpt2-medium-fp8 run fp8_$r REPLICANN_X=0 || exit 1
  M=gpt2-medium-fp8 run fp8head_$r REPLICANN_FP8_HEAD=1 || exit 1
done
REPLICANN_FP8_HEAD=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_5o -o run -- python3 bench.py --model gpt2-medium-fp8 --steps 3 --warmup 2 > gpurun_out/r5o_prof.log 2>&1 || { echo "prof failed"; exit 1; }
python scripts/prof_steps.py gpurun_out/prof_5o/run_kernel_trace.csv --steps 3 > gpurun_out/r5o_steps_m8.txt 2>&1
rm -rf gpurun_out/prof_5o
head -30 gpurun_out/r5o_steps_m8.txt | cut -c1-150
REPLICANN_FP8_HEAD=1 timeout -k 10 400 python -u scripts/fp8_trajectory.py 50 16 1e-4 > gpurun_out/r5o_traj_head.jsonl 2> gpurun_out/r5o_traj_head.err || { echo "trajectory failed"; tail -5 gpurun_out/r5o_traj_head.err; exit 1; }
echo "traj head: $(grep summary gpurun_out/r5o_traj_head.jsonl)"
