#!/bin/bash
# round 5: the attention forward writes the fp8 output projection's e4m3 input (REPLICANN_FP8_ATTN_O8): tests (bitwise vs
# the quantisation pass, a whole fp8 step bitwise), attention / fp8 suites, then GPT-2-medium-fp8 off / on alternating and
# the GPT-2-small headline (its attention kernel is instruction-for-instruction unchanged).
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
PT="python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 500 $PT tests/test_fp8_ln_q8_gpu.py tests/test_fp8_head_gpu.py tests/test_fp8_wgrad_gpu.py tests/test_fp8_inference_gpu.py tests/test_fp8_state.py tests/test_models.py tests/test_determinism_gpu.py tests/test_ops_gpu.py -k "fp8 or attention or attn or gpt2 or determin" > gpurun_out/r5o8_tests.log 2>&1; rc=$?
echo "=== tests rc=$rc"; grep -E "FAILED|Error|passed|failed" gpurun_out/r5o8_tests.log | tail -6
[ $rc -eq 0 ] || exit $rc
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 240 python -u bench.py --model gpt2-medium-fp8 --steps 6 --warmup 3 > gpurun_out/r5o8_$tag.log 2>&1 || { echo "bench $tag failed"; tail -5 gpurun_out/r5o8_$tag.log; exit 1; }
  echo "$tag: $(grep -o '"value": [0-9.]*' gpurun_out/r5o8_$tag.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5o8_$tag.log)"
}
for r in 1 2; do
  run off_$r REPLICANN_FP8_ATTN_O8=0 || exit 1
  run on_$r REPLICANN_X=0 || exit 1
done
timeout -k 10 300 python -u bench.py > gpurun_out/r5o8_gpt2s.log 2>&1 || { echo "gpt2s failed"; exit 1; }
echo "gpt2-small: $(grep -o '"value": [0-9.]*' gpurun_out/r5o8_gpt2s.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5o8_gpt2s.log)"
