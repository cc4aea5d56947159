#!/bin/bash
# round 4 (call N): PMC counters of every kernel in the GPT-2-small step at HEAD (MFMA busy, wait split,
# LDS conflicts, VALU / MFMA instruction mix, HBM fetch) — 3 rocprofv3 passes of 2 steps each; then the
# committed GEMM tuning tables vs a fresh runtime tuning (REPLICANN_GEMM_TABLES=0) for GPT-2-small and
# ViT-B/16 (the fresh run goes last, so gpurun_out/gemm_tuning_<model>.json holds the new picks).
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
fault() { grep -q "illegal memory access\|hipErrorIllegalAddress\|HSA_STATUS_ERROR\|Memory access fault" "$1"; }
# first: the fused ViT token join (new kernels) against fp32, and the ViT models on the GPU
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_ops_gpu.py tests/test_convergence_gpu.py tests/test_models.py -k "vit or embedding or attention" > gpurun_out/n_tests.log 2>&1; rc=$?
echo "=== n_tests rc=$rc $(grep -E 'passed|failed' gpurun_out/n_tests.log | tail -1)"; grep -E "FAILED" gpurun_out/n_tests.log | head
fault gpurun_out/n_tests.log && exit 2; [ $rc -ne 0 ] && exit 1
timeout -k 10 1000 bash scripts/pmc_step.sh "--steps 2 --warmup 1" gpt2s > gpurun_out/n_pmc.log 2>&1 || { echo "pmc failed"; tail -5 gpurun_out/n_pmc.log; exit 1; }
python scripts/pmc_summary.py gpurun_out/pmc_step/gpt2s*_counter_collection.csv > gpurun_out/pmc_step_summary.txt 2>&1
head -60 gpurun_out/pmc_step_summary.txt | cut -c1-260
for m in gpt2-small vit-b16; do
  for r in 1 2; do
    for tb in 1 0; do
      REPLICANN_GEMM_TABLES=$tb timeout -k 10 400 python bench.py --model $m --steps 8 --warmup 3 > gpurun_out/n_tab_${m}_${tb}_$r.log 2>&1 || { echo "bench $m failed"; exit 1; }
      echo "$m tables=$tb r$r: $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/n_tab_${m}_${tb}_$r.log | tr '\n' ' ')"
    done
  done
done
exit 0
