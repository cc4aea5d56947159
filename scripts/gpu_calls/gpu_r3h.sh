#!/bin/bash
# round 3: persistent-GEMM start skew between phase groups (epilogue store-burst spreading)
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
out=gpurun_out/skew.jsonl; : > $out
for sk in 0 1500 3000 6500 13000; do
  for s in "65536 50304 768 nt" "65536 2304 768 nt" "65536 3072 768 nt --act 5"; do
    REPLICANN_GEMM_SKEW=$sk REPLICANN_GEMM_SKEW_MIN=1 timeout -k 10 120 python scripts/gemm_one.py $s --iters 30 > gpurun_out/one.log 2>&1 || { cat gpurun_out/one.log; exit 1; }
    echo "{\"skew\": $sk, \"r\": $(grep '^{' gpurun_out/one.log)}" | tee -a $out
  done
done
