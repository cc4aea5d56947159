#!/bin/bash
# round 4 (call M): attention forward + backward skip dead (group, 16-row block) pieces of masked tiles (causal
# diagonal upper blocks, ragged tails): fp32-reference + determinism tests, then A/B against the previous
# library (ab/_C_prev.so) at GPT-2-small (causal T = 1024) and ViT-B/16 (T = 197) shapes and on both steps.
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
fault() { grep -q "illegal memory access\|hipErrorIllegalAddress\|HSA_STATUS_ERROR\|Memory access fault" "$1"; }
PT="python -u -m pytest -q --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 400 $PT tests/test_ops_gpu.py tests/test_determinism_gpu.py tests/test_reference_parity_gpu.py -k "attention or attn or determin or parity or grads" > gpurun_out/m_tests.log 2>&1; rc=$?
echo "=== m_tests rc=$rc $(grep -E 'passed|failed' gpurun_out/m_tests.log | tail -1)"; grep -E "FAILED|^E  .*Error" gpurun_out/m_tests.log | head
fault gpurun_out/m_tests.log && exit 2; [ $rc -ne 0 ] && exit 1
lib() { if [ $1 = prev ]; then export REPLICANN_SO=ab/_C_prev.so; else unset REPLICANN_SO; fi; }
for r in 1 2 3; do
  for l in prev new; do
    lib $l
    timeout -k 10 120 python scripts/attn_ab.py 64 --rounds 3 > gpurun_out/m_gpt_${l}_$r.log 2>&1 || { echo "attn_ab failed"; exit 1; }
    timeout -k 10 120 python scripts/attn_ab.py 512 --T 197 --noncausal --rounds 3 > gpurun_out/m_vit_${l}_$r.log 2>&1 || { echo "attn_ab vit failed"; exit 1; }
    echo "$l r$r gpt: $(grep -o '"op": "[a-z_]*".*"tflops": [0-9.]*' gpurun_out/m_gpt_${l}_$r.log | sed 's/, "B".*"ms"/ ms/' | tr '\n' ' ')  vit: $(grep -o '"op": "[a-z_]*".*"tflops": [0-9.]*' gpurun_out/m_vit_${l}_$r.log | sed 's/, "B".*"ms"/ ms/' | tr '\n' ' ')"
  done
done
unset REPLICANN_SO
for l in prev new; do
  lib $l
  timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/m_kt_$l -o run -- python3 scripts/attn_ab.py 64 --rounds 2 > /dev/null 2>&1 || { echo "trace failed"; exit 1; }
  echo "$l kernels:"; python -c "
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'attn' in r['Name']: print('  %8.1f us x%s  %s' % (float(r['AverageNs'])/1e3, r['Calls'], r['Name'][:80]))
" gpurun_out/m_kt_$l/run_kernel_stats.csv
done
for r in 1 2; do
  for l in prev new; do
    lib $l
    timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/m_bench_${l}_$r.log 2>&1 || { echo "bench failed"; exit 1; }
    timeout -k 10 300 python bench.py --model vit-b16 --steps 8 --warmup 3 > gpurun_out/m_vitb_${l}_$r.log 2>&1 || { echo "vit bench failed"; exit 1; }
    echo "bench $l r$r: gpt2s $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/m_bench_${l}_$r.log | tr '\n' ' ') vit $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/m_vitb_${l}_$r.log | tr '\n' ' ')"
  done
done
exit 0
