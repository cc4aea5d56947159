#!/bin/bash
# round 3: persistent GEMM fixed per-launch cost (M sweep, graph-replayed) + nt logits store check
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python scripts/gemm_msweep.py > gpurun_out/msweep.jsonl 2> gpurun_out/msweep.err || { tail -20 gpurun_out/msweep.err; exit 1; }
cat gpurun_out/msweep.jsonl
timeout -k 10 120 python scripts/gemm_one.py 65536 50304 768 nt --iters 30 && \
REPLICANN_GEMM_ST_NT=0 timeout -k 10 120 python scripts/gemm_one.py 65536 50304 768 nt --iters 30
