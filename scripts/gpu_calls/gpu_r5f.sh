#!/bin/bash
# round 5 (call F): cfg 11 after the RES0 wait fix + next-tile residual prefetch, and its fp8 data-gradient
# path (MN-contiguous B via tr_b8): tests, A/B, fp8 backward A/B vs the older dgrad kernel, and the
# all-L2-hit ablation (DBG 8: every tile's DMA reads tile (0,0)'s rows) against DBG 0 / 2.
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
PT="python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 400 $PT tests/test_gemm_w1_gpu.py tests/test_fp8_inference_gpu.py tests/test_fp8_wgrad_gpu.py tests/test_ops_gpu.py -k "fp8 or w1" > gpurun_out/r5f_tests.log 2>&1; rc=$?
echo "=== tests rc=$rc"; grep -E "FAILED|passed|failed" gpurun_out/r5f_tests.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/w1_ab.py --rounds 5 > gpurun_out/r5f_w1_ab.log 2>&1 || exit 1
grep -E '_res|fp8' gpurun_out/r5f_w1_ab.log | cut -c1-200
for k in 9 11; do
  REPLICANN_FP8_GEMM=$k timeout -k 10 200 python -u scripts/fp8_bwd_ab.py 65536 3 > gpurun_out/r5f_bwd_ab_$k.log 2>&1 || { echo "bwd ab $k failed"; exit 1; }
  echo "== fp8 dgrad kernel $k"; grep '^{' gpurun_out/r5f_bwd_ab_$k.log | cut -c1-260
done
for d in 0 8 2; do
  for spec in "65536 768 3072 nt --cfg 11" "65536 2304 768 nt --cfg 11 --bias" "65536 3072 1024 nt --fp8 11" "65536 4096 1024 nt --fp8 11"; do
    REPLICANN_W1_DBG=$d timeout -k 10 60 python3 scripts/gemm_one.py $spec --iters 30 | sed "s/^/dbg=$d /" || exit 1
  done
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r5f_ablate.log
