#!/bin/bash
# round 5 (call C): cfg 11 with the post-epilogue store allowance: tests, graph A/B vs cfg 9 / older fp8
# kernels, nt-store ablation, L2 (TCC) counters.
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
PT="python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 400 $PT tests/test_gemm_w1_gpu.py tests/test_fp8_inference_gpu.py tests/test_ops_gpu.py -k "fp8 or w1" > gpurun_out/r5c_tests.log 2>&1; rc=$?
echo "=== tests rc=$rc"; grep -E "FAILED|passed|failed" gpurun_out/r5c_tests.log | tail -8
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u scripts/w1_ab.py --rounds 5 > gpurun_out/r5c_w1_ab.log 2>&1 || exit 1
grep '^{' gpurun_out/r5c_w1_ab.log | cut -c1-200
for d in 0 4; do
  for spec in "65536 768 3072 nt --cfg 11" "65536 2304 768 nt --cfg 11 --bias" "65536 3072 1024 nt --fp8 11" "65536 4096 1024 nt --fp8 11"; do
    REPLICANN_W1_DBG=$d timeout -k 10 60 python3 scripts/gemm_one.py $spec --iters 30 | sed "s/^/dbg=$d /" || exit 1
  done
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r5c_ablate.log
rc=${PIPESTATUS[0]}; [ $rc -eq 0 ] || exit $rc
i=0
for spec in "65536 768 3072 nt --cfg 11" "65536 768 3072 nt --cfg 9" "65536 3072 1024 nt --fp8 11" "65536 3072 1024 nt --fp8 9"; do
  i=$((i + 1))
  timeout -s KILL 60 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum GRBM_GUI_ACTIVE \
     --kernel-trace --output-format csv -d gpurun_out/pmc_tcc -o run${i}_c -- python3 scripts/gemm_one.py $spec --iters 3 > /dev/null 2>&1 || { echo "pmc $i failed"; exit 1; }
done
python3 scripts/pmc_summary.py gpurun_out/pmc_tcc/*_counter_collection.csv --match gemm > gpurun_out/r5c_tcc.txt 2>&1; cut -c1-60,100-400 gpurun_out/r5c_tcc.txt
