#!/bin/bash
# round 5 (call A): first run of the one-wave-per-SIMD GEMM (cfg 11): numerics vs fp32, then A/B vs cfg 9.
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 90 python -u -c "
import torch; from replicann_amd import ops
for (M,N,K) in [(256,256,128),(512,512,256),(4096,1024,768)]:
    a=torch.randn(M,K,device='cuda').bfloat16(); b=(torch.randn(N,K,device='cuda')*0.05).bfloat16()
    o=ops.gemm(a,b,tb=True,cfg=11); torch.cuda.synchronize()
    r=a.float()@b.float().t(); print(M,N,K,((o.float()-r).norm()/r.norm()).item(), flush=True)
" > gpurun_out/r5a_smoke.log 2>&1; rc=$?; cat gpurun_out/r5a_smoke.log; [ $rc -eq 0 ] || exit $rc
PT="python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 500 $PT tests/test_gemm_w1_gpu.py > gpurun_out/r5a_w1_test.log 2>&1; rc=$?
echo "=== w1 tests rc=$rc"; grep -E "PASSED|FAILED|Error|error|passed|failed" gpurun_out/r5a_w1_test.log | tail -40
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/w1_ab.py --rounds 5 > gpurun_out/r5a_w1_ab.log 2>&1; rc=$?
echo "=== w1_ab rc=$rc"; cat gpurun_out/r5a_w1_ab.log | cut -c1-200
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 $PT tests/test_ops_gpu.py -k "fp8" tests/test_fp8_wgrad_gpu.py tests/test_fp8_inference_gpu.py > gpurun_out/r5a_fp8_tests.log 2>&1; rc=$?
echo "=== fp8 tests rc=$rc"; grep -E "FAILED|passed|failed" gpurun_out/r5a_fp8_tests.log | tail -15
exit $rc
