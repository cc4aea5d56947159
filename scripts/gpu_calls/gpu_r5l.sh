#!/bin/bash
# round 5 (call L): attention backward emitting e5m2 dQKV for the fp8 c_attn (bf16 dQKV skipped when c_attn takes
# both gradients in fp8); unrolled e5m2 / gelu quantisers.  Tests, GPT-2-medium bf16 / fp8 / fp8 with
# REPLICANN_FP8_ATTN_Q8=0 alternating, breakdown, trajectory.
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
PT="python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $PT tests/test_fp8_wgrad_gpu.py tests/test_fp8_inference_gpu.py tests/test_determinism_gpu.py tests/test_ops_gpu.py -k "fp8 or attn or attention or gelu or act_mul or determin" > gpurun_out/r5l_tests.log 2>&1; rc=$?
echo "=== tests rc=$rc"; grep -E "FAILED|passed|failed" gpurun_out/r5l_tests.log | tail -8
[ $rc -eq 0 ] || exit $rc
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 240 python -u bench.py --model ${M} --steps 6 --warmup 3 > gpurun_out/r5l_$tag.log 2>&1 || { echo "bench $tag failed"; tail -5 gpurun_out/r5l_$tag.log; exit 1; }
  echo "$tag: $(grep -o '"value": [0-9.]*' gpurun_out/r5l_$tag.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5l_$tag.log) $(grep -o '"loss_first_last": [^]]*]' gpurun_out/r5l_$tag.log)"
}
for r in 1 2; do
  M=gpt2-medium run bf16_$r REPLICANN_X=0 || exit 1
  M=gpt2-medium-fp8 run fp8_$r REPLICANN_X=0 || exit 1
  M=gpt2-medium-fp8 run fp8noq8_$r REPLICANN_FP8_ATTN_Q8=0 || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_5l -o run -- python3 bench.py --model gpt2-medium-fp8 --steps 3 --warmup 2 > gpurun_out/r5l_prof.log 2>&1 || { echo "prof failed"; exit 1; }
python scripts/prof_steps.py gpurun_out/prof_5l/run_kernel_trace.csv --steps 3 > gpurun_out/r5l_steps_m8.txt 2>&1
rm -rf gpurun_out/prof_5l
head -26 gpurun_out/r5l_steps_m8.txt | cut -c1-150
timeout -k 10 500 python -u scripts/fp8_trajectory.py 50 16 1e-4 > gpurun_out/r5l_traj.jsonl 2> gpurun_out/r5l_traj.err || { echo "trajectory failed"; tail -5 gpurun_out/r5l_traj.err; exit 1; }
grep summary gpurun_out/r5l_traj.jsonl
