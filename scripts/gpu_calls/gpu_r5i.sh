#!/bin/bash
# round 5 (call I): the fused fp8 MLP backward (c_proj fp8 dgrad + GELU backward fused into dH's e5m2 pass):
# tests, GPT-2-medium bf16 / fp8 (fused) / fp8 (REPLICANN_FP8_MLP_FUSE=0) alternating, breakdown, trajectory.
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
PT="python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 400 $PT tests/test_fp8_wgrad_gpu.py tests/test_fp8_inference_gpu.py tests/test_gemm_w1_gpu.py tests/test_ops_gpu.py -k "fp8 or w1 or mlp" > gpurun_out/r5i_tests.log 2>&1; rc=$?
echo "=== tests rc=$rc"; grep -E "FAILED|passed|failed" gpurun_out/r5i_tests.log | tail -8
[ $rc -eq 0 ] || exit $rc
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 240 python -u bench.py --model ${M} --steps 6 --warmup 3 > gpurun_out/r5i_$tag.log 2>&1 || { echo "bench $tag failed"; tail -5 gpurun_out/r5i_$tag.log; exit 1; }
  echo "$tag: $(grep -o '"value": [0-9.]*' gpurun_out/r5i_$tag.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5i_$tag.log) $(grep -o '"loss_first_last": [^]]*]' gpurun_out/r5i_$tag.log)"
}
for r in 1 2; do
  M=gpt2-medium run bf16_$r REPLICANN_X=0 || exit 1
  M=gpt2-medium-fp8 run fp8fused_$r REPLICANN_X=0 || exit 1
  M=gpt2-medium-fp8 run fp8unfused_$r REPLICANN_FP8_MLP_FUSE=0 || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_5i -o run -- python3 bench.py --model gpt2-medium-fp8 --steps 3 --warmup 2 > gpurun_out/r5i_prof.log 2>&1 || { echo "prof failed"; exit 1; }
python scripts/prof_steps.py gpurun_out/prof_5i/run_kernel_trace.csv --steps 3 > gpurun_out/r5i_steps_m8.txt 2>&1
rm -rf gpurun_out/prof_5i
head -30 gpurun_out/r5i_steps_m8.txt | cut -c1-150
timeout -k 10 500 python -u scripts/fp8_trajectory.py 50 16 1e-4 > gpurun_out/r5i_traj.jsonl 2> gpurun_out/r5i_traj.err || { echo "trajectory failed"; tail -5 gpurun_out/r5i_traj.err; exit 1; }
grep summary gpurun_out/r5i_traj.jsonl
