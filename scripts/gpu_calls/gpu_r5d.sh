#!/bin/bash
# round 5 (call D): tests; cfg 11 residual A/B; GPT-2-medium bf16 vs fp8 (cfg 11 the default fp8 forward
# for c_attn / c_proj / MLP c_proj); stock-PyTorch baselines on the same box (verdict r4 item 8).
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
PT="python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 400 $PT tests/test_gemm_w1_gpu.py tests/test_fp8_inference_gpu.py tests/test_fp8_wgrad_gpu.py tests/test_ops_gpu.py -k "fp8 or w1" > gpurun_out/r5d_tests.log 2>&1; rc=$?
echo "=== tests rc=$rc"; grep -E "FAILED|passed|failed" gpurun_out/r5d_tests.log | tail -8
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u scripts/w1_ab.py --rounds 5 > gpurun_out/r5d_w1_ab.log 2>&1 || exit 1
grep '_res' gpurun_out/r5d_w1_ab.log | cut -c1-200
for r in 1 2; do
  for m in gpt2-medium gpt2-medium-fp8; do
    timeout -k 10 240 python -u bench.py --model $m --steps 6 --warmup 3 > gpurun_out/r5d_bench_${m}_$r.log 2>&1 || { echo "bench $m failed"; tail -5 gpurun_out/r5d_bench_${m}_$r.log; exit 1; }
    echo "$m run $r: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5d_bench_${m}_$r.log)"
  done
done
for m in gpt2-small vit-b16 resnet18; do
  timeout -k 10 240 python -u scripts/bench_stock_torch.py --model $m --steps 10 --warmup 3 > gpurun_out/r5d_stock_$m.log 2>&1 || { echo "stock $m failed"; tail -5 gpurun_out/r5d_stock_$m.log; exit 1; }
  echo "stock $m: $(grep '^{' gpurun_out/r5d_stock_$m.log | cut -c1-220)"
done
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r5d_bench_gpt2s.log 2>&1; echo "gpt2-small native: $(grep -o '"value": [0-9.]*, "unit": "[^"]*", "n_gpus": 1, "steps": 20, "warmup": 5, "ms_per_step": [0-9.]*' gpurun_out/r5d_bench_gpt2s.log)"
