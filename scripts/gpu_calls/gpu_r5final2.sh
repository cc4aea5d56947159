#!/bin/bash
# round 5 closing run after the LayerNorm-backward e5m2 change: full pytest -m gpu, smoke(), GPT-2-small against
# abso/_C_old.so (the tree before this round's attention / conv / LayerNorm kernel changes) alternating, the other
# bench configs, then the conv3x3 PMC passes (scripts/gpu_calls/gpu_r5pmc.sh).
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r5f2_gpu_tests.log 2>&1; rc=$?
echo "=== gpu tests rc=$rc"; grep -E "FAILED|Error|passed|failed" gpurun_out/r5f2_gpu_tests.log | tail -6
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5f2_smoke.log 2>&1 || { echo "smoke failed"; tail -5 gpurun_out/r5f2_smoke.log; exit 1; }
tail -1 gpurun_out/r5f2_smoke.log
for r in 1 2; do
  REPLICANN_SO=abso/_C_old.so timeout -k 10 300 python -u bench.py > gpurun_out/r5f2_old_$r.log 2>&1 || { echo "old bench failed"; tail -3 gpurun_out/r5f2_old_$r.log; exit 1; }
  timeout -k 10 300 python -u bench.py > gpurun_out/r5f2_new_$r.log 2>&1 || { echo "bench failed"; tail -3 gpurun_out/r5f2_new_$r.log; exit 1; }
  echo "gpt2-small r$r old: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5f2_old_$r.log)  new: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5f2_new_$r.log)"
done
tail -1 gpurun_out/r5f2_new_2.log
for M in gpt2-medium gpt2-medium-fp8 vit-b16 resnet18; do
  timeout -k 10 300 python -u bench.py --model $M --steps 10 --warmup 3 > gpurun_out/r5f2_$M.log 2>&1 || { echo "bench $M failed"; tail -5 gpurun_out/r5f2_$M.log; exit 1; }
  echo "$M: $(grep -o '"value": [0-9.]*' gpurun_out/r5f2_$M.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5f2_$M.log)"
done
bash scripts/gpu_calls/gpu_r5pmc.sh
