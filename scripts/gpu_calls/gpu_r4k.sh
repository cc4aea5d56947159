#!/bin/bash
# round 4 (call K): attention backward with the dP accumulators started at −δ (one multiply for dS) and
# masked scores sent to −inf before the exp (one select per element): fp32-reference + determinism
# tests, then A/B against the previous library (ab/_C_prev.so = HEAD before the change) on GPT-2-small
# shapes and on the step.
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
fault() { grep -q "illegal memory access\|hipErrorIllegalAddress\|HSA_STATUS_ERROR\|Memory access fault" "$1"; }
PT="python -u -m pytest -q --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 400 $PT tests/test_ops_gpu.py tests/test_determinism_gpu.py tests/test_reference_parity_gpu.py -k "attention or attn or determin or parity or grads" > gpurun_out/k_tests.log 2>&1; rc=$?
echo "=== k_tests rc=$rc $(grep -E 'passed|failed' gpurun_out/k_tests.log | tail -1)"; grep -E "FAILED|^E  .*Error" gpurun_out/k_tests.log | head
fault gpurun_out/k_tests.log && exit 2; [ $rc -ne 0 ] && exit 1
for r in 1 2 3; do
  for lib in prev new; do
    if [ $lib = prev ]; then export REPLICANN_SO=ab/_C_prev.so; else unset REPLICANN_SO; fi
    timeout -k 10 120 python scripts/attn_ab.py 64 --rounds 3 > gpurun_out/k_attn_${lib}_$r.log 2>&1 || { echo "attn_ab $lib failed"; exit 1; }
    echo "$lib r$r: $(grep -o '"op": "[a-z_]*".*"tflops": [0-9.]*' gpurun_out/k_attn_${lib}_$r.log | sed 's/, "B".*"ms"/ ms/' | tr '\n' ' ')"
  done
done
unset REPLICANN_SO
for lib in prev new; do
  if [ $lib = prev ]; then export REPLICANN_SO=ab/_C_prev.so; else unset REPLICANN_SO; fi
  timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/k_kt_$lib -o run -- python3 scripts/attn_ab.py 64 --rounds 2 > /dev/null 2>&1 || { echo "trace $lib failed"; exit 1; }
  echo "$lib kernels:"; python -c "
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'attn' in r['Name']: print('  %8.1f us x%s  %s' % (float(r['AverageNs'])/1e3, r['Calls'], r['Name'][:80]))
" gpurun_out/k_kt_$lib/run_kernel_stats.csv
done
unset REPLICANN_SO
for r in 1 2; do
  for lib in prev new; do
    if [ $lib = prev ]; then export REPLICANN_SO=ab/_C_prev.so; else unset REPLICANN_SO; fi
    timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/k_bench_${lib}_$r.log 2>&1 || { echo "bench failed"; exit 1; }
    echo "bench $lib r$r: $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/k_bench_${lib}_$r.log | tr '\n' ' ')"
  done
done
exit 0
