#!/bin/bash
# round 6 final validation (resident attention + 8-wave causal forward): full pytest -m gpu, smoke(), every bench config (GPT-2 small / medium / medium-fp8, ViT-B/16,
# ResNet-18) on one box.
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r6fin3_gpu_tests.log 2>&1; rc=$?
echo "=== gpu tests rc=$rc"; grep -E "FAILED|Error|passed|failed" gpurun_out/r6fin3_gpu_tests.log | tail -6
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r6fin3_smoke.log 2>&1 || { echo "smoke failed"; tail -5 gpurun_out/r6fin3_smoke.log; exit 1; }
tail -1 gpurun_out/r6fin3_smoke.log
timeout -k 10 300 python -u bench.py > gpurun_out/r6fin3_bench.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r6fin3_bench.log; exit 1; }
tail -1 gpurun_out/r6fin3_bench.log
for M in gpt2-medium gpt2-medium-fp8 vit-b16 resnet18; do
  timeout -k 10 300 python -u bench.py --model $M --steps 10 --warmup 3 > gpurun_out/r6fin3_$M.log 2>&1 || { echo "bench $M failed"; tail -5 gpurun_out/r6fin3_$M.log; exit 1; }
  echo "$M: $(grep -o '"value": [0-9.]*' gpurun_out/r6fin3_$M.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r6fin3_$M.log)"
done
