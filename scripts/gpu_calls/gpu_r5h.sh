#!/bin/bash
# round 5 (call H): cfg 11 tile-walk group height (REPLICANN_W1_GROUP: tile-rows per group) vs L2 reuse.
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gemm_w1_gpu.py > gpurun_out/r5h_tests.log 2>&1; rc=$?
echo "=== w1 tests rc=$rc $(tail -1 gpurun_out/r5h_tests.log)"; [ $rc -eq 0 ] || exit $rc
for g in 8 4 2 11 16 32 8; do
  for spec in "65536 768 3072 nt --cfg 11" "65536 2304 768 nt --cfg 11 --bias" "65536 3072 1024 nt --fp8 11" "65536 4096 1024 nt --fp8 11"; do
    REPLICANN_W1_GROUP=$g timeout -k 10 60 python3 scripts/gemm_one.py $spec --iters 30 | sed "s/^/group=$g /" || exit 1
  done
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r5h_group.log
rc=${PIPESTATUS[0]}; [ $rc -eq 0 ] || exit $rc
# PMC of the fp8 forward bodies (verdict r4 item 1: MFMA busy and LDS instructions per MFMA)
i=0
for spec in "65536 3072 1024 nt --fp8 11" "65536 3072 1024 nt --fp8 0" "65536 4096 1024 nt --fp8 11" "65536 4096 1024 nt --fp8 0"; do
  i=$((i + 1))
  timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_MFMA SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE \
     --kernel-trace --output-format csv -d gpurun_out/pmc_5h -o run${i} -- python3 scripts/gemm_one.py $spec --iters 3 > /dev/null 2>&1 || { echo "pmc $i failed"; exit 1; }
done
python3 scripts/pmc_summary.py gpurun_out/pmc_5h/*_counter_collection.csv --match gemm > gpurun_out/r5h_pmc.txt 2>&1; cut -c1-60,100-500 gpurun_out/r5h_pmc.txt
# GPT-2-medium-fp8 step breakdown with the fp8 backward on (REPLICANN_FP8_DGRAD/WGRAD=1)
REPLICANN_FP8_DGRAD=1 REPLICANN_FP8_WGRAD=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_5h -o run -- python3 bench.py --model gpt2-medium-fp8 --steps 3 --warmup 2 > gpurun_out/r5h_prof.log 2>&1 || { echo "prof failed"; exit 1; }
python scripts/prof_steps.py gpurun_out/prof_5h/run_kernel_trace.csv --steps 3 > gpurun_out/r5h_steps_m8all.txt 2>&1
rm -rf gpurun_out/prof_5h
head -40 gpurun_out/r5h_steps_m8all.txt | cut -c1-150
