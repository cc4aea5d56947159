#!/bin/bash
# round 5 (call T): as call S, without the dQ −δ accumulator start (packed exponent FMAs only) — old vs new.
# (abso/_C_old.so = HEAD's attention) vs the new one alternating: attention microbench and GPT-2-small step.
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
PT="python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 400 $PT tests/test_ops_gpu.py -k "attention or attn" tests/test_determinism_gpu.py tests/test_fp8_wgrad_gpu.py tests/test_reference_parity_gpu.py > gpurun_out/r5t_tests.log 2>&1; rc=$?
echo "=== tests rc=$rc"; grep -E "FAILED|Error|passed|failed" gpurun_out/r5t_tests.log | tail -6
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  REPLICANN_SO=abso/_C_old.so timeout -k 10 200 python -u scripts/attn_ab.py 64 > gpurun_out/r5t_attn_old_$r.log 2>&1 || { echo "attn old failed"; tail -5 gpurun_out/r5t_attn_old_$r.log; exit 1; }
  timeout -k 10 200 python -u scripts/attn_ab.py 64 > gpurun_out/r5t_attn_new_$r.log 2>&1 || { echo "attn new failed"; tail -5 gpurun_out/r5t_attn_new_$r.log; exit 1; }
  echo "old_$r:"; cat gpurun_out/r5t_attn_old_$r.log | grep "{"; echo "new_$r:"; cat gpurun_out/r5t_attn_new_$r.log | grep "{"
done
for r in 1 2; do
  REPLICANN_SO=abso/_C_old.so timeout -k 10 200 python -u bench.py > gpurun_out/r5t_b_old_$r.log 2>&1 || { echo "bench old failed"; tail -5 gpurun_out/r5t_b_old_$r.log; exit 1; }
  timeout -k 10 200 python -u bench.py > gpurun_out/r5t_b_new_$r.log 2>&1 || { echo "bench new failed"; tail -5 gpurun_out/r5t_b_new_$r.log; exit 1; }
  echo "gpt2s old_$r: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5t_b_old_$r.log)  new_$r: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5t_b_new_$r.log)"
done
