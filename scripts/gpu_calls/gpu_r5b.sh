#!/bin/bash
# round 5 (call B): fp8 tests after the power-of-two scale change; cfg-11 timing ablations (DBG: stores /
# DMA out of range) and PMC of cfg 11 vs cfg 9 on steady-state (K = 3072) and K = 768/1024 shapes.
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
PT="python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 400 $PT tests/test_gemm_w1_gpu.py tests/test_ops_gpu.py -k "fp8 or w1" tests/test_fp8_wgrad_gpu.py tests/test_fp8_inference_gpu.py > gpurun_out/r5b_fp8_tests.log 2>&1; rc=$?
echo "=== fp8 tests rc=$rc"; grep -E "FAILED|passed|failed" gpurun_out/r5b_fp8_tests.log | tail -15
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc   # (assertion failures: go on to the timings)
for d in 0 1 2 3; do
  for spec in "65536 768 3072 nt --cfg 11" "65536 2304 768 nt --cfg 11 --bias" "65536 3072 1024 nt --fp8 11" "65536 4096 1024 nt --fp8 11"; do
    REPLICANN_W1_DBG=$d timeout -k 10 60 python3 scripts/gemm_one.py $spec --iters 30 | sed "s/^/dbg=$d /" || exit 1
  done
done 2>&1 | tee gpurun_out/r5b_ablate.log | grep -v amdgpu.ids
rc=${PIPESTATUS[0]}; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 bash scripts/pmc_w1.sh gpurun_out/pmc_w1 "65536 768 3072 nt --cfg 11" "65536 768 3072 nt --cfg 9" \
  "65536 3072 1024 nt --fp8 11" "65536 3072 1024 nt --fp8 9" "65536 2304 768 nt --cfg 11 --bias" "65536 2304 768 nt --cfg 9 --bias" > gpurun_out/r5b_pmc.log 2>&1; rc=$?
echo "=== pmc rc=$rc"; grep -v amdgpu.ids gpurun_out/r5b_pmc.log | tail -8
python3 scripts/pmc_summary.py gpurun_out/pmc_w1/*_counter_collection.csv > gpurun_out/r5b_pmc_summary.txt 2>&1; cut -c1-400 gpurun_out/r5b_pmc_summary.txt
exit $rc
