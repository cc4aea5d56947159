#!/bin/bash
# round 5 (call M): grid-strided amax reduce for the attention e5m2 dQKV; gelu_q8 on a larger grid.
# fp8 tests, GPT-2-medium bf16 / fp8 alternating, breakdown; GPT-2-small bench.
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
PT="python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 400 $PT tests/test_fp8_wgrad_gpu.py tests/test_fp8_inference_gpu.py > gpurun_out/r5m_tests.log 2>&1; rc=$?
echo "=== tests rc=$rc"; grep -E "FAILED|passed|failed" gpurun_out/r5m_tests.log | tail -4
[ $rc -eq 0 ] || exit $rc
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 240 python -u bench.py --model ${M} --steps 6 --warmup 3 > gpurun_out/r5m_$tag.log 2>&1 || { echo "bench $tag failed"; tail -5 gpurun_out/r5m_$tag.log; exit 1; }
  echo "$tag: $(grep -o '"value": [0-9.]*' gpurun_out/r5m_$tag.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5m_$tag.log)"
}
for r in 1 2; do
  M=gpt2-medium run bf16_$r REPLICANN_X=0 || exit 1
  M=gpt2-medium-fp8 run fp8_$r REPLICANN_X=0 || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_5m -o run -- python3 bench.py --model gpt2-medium-fp8 --steps 3 --warmup 2 > gpurun_out/r5m_prof.log 2>&1 || { echo "prof failed"; exit 1; }
python scripts/prof_steps.py gpurun_out/prof_5m/run_kernel_trace.csv --steps 3 > gpurun_out/r5m_steps_m8.txt 2>&1
rm -rf gpurun_out/prof_5m
head -22 gpurun_out/r5m_steps_m8.txt | cut -c1-150
timeout -k 10 200 python -u bench.py > gpurun_out/r5m_gpt2s.log 2>&1; echo "gpt2-small: $(grep -o '"value": [0-9.]*' gpurun_out/r5m_gpt2s.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5m_gpt2s.log)"
