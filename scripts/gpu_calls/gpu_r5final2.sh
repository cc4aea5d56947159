#!/bin/bash
# round 5 closing run after the LayerNorm-backward e5m2 change: full pytest -m gpu, smoke(), every bench config,
# then the conv3x3 PMC passes (scripts/gpu_calls/gpu_r5pmc.sh).  (The A/B against abso/_C_old.so is gone: that
# library predates the layernorm_bwd schema change; the bf16 LayerNorm-backward code is unchanged instruction for
# instruction — the Q8 variant is a separate instantiation.)
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r5f2_gpu_tests.log 2>&1; rc=$?
echo "=== gpu tests rc=$rc"; grep -E "FAILED|Error|passed|failed" gpurun_out/r5f2_gpu_tests.log | tail -6
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5f2_smoke.log 2>&1 || { echo "smoke failed"; tail -5 gpurun_out/r5f2_smoke.log; exit 1; }
tail -1 gpurun_out/r5f2_smoke.log
timeout -k 10 300 python -u bench.py > gpurun_out/r5f2_new_1.log 2>&1 || { echo "bench failed"; tail -3 gpurun_out/r5f2_new_1.log; exit 1; }
timeout -k 10 300 python -u bench.py > gpurun_out/r5f2_new_2.log 2>&1 || { echo "bench failed"; tail -3 gpurun_out/r5f2_new_2.log; exit 1; }
echo "gpt2-small: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5f2_new_1.log) / $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5f2_new_2.log)"
tail -1 gpurun_out/r5f2_new_2.log
for M in gpt2-medium gpt2-medium-fp8 vit-b16 resnet18; do
  timeout -k 10 300 python -u bench.py --model $M --steps 10 --warmup 3 > gpurun_out/r5f2_$M.log 2>&1 || { echo "bench $M failed"; tail -5 gpurun_out/r5f2_$M.log; exit 1; }
  echo "$M: $(grep -o '"value": [0-9.]*' gpurun_out/r5f2_$M.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5f2_$M.log)"
done
bash scripts/gpu_calls/gpu_r5pmc.sh
