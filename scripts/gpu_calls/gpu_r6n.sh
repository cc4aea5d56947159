#!/bin/bash
# round 6 call N: whole-row XCD bands for cfg 9 (REPLICANN_GEMM_BAND=1): GEMM GPU tests with it on, per-shape A/B, bench A/B
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
REPLICANN_GEMM_BAND=1 timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py -k "gemm or linear or mlp" tests/test_gemm_sched_gpu.py tests/test_determinism_gpu.py > gpurun_out/r6n_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r6n_tests.log; [ $rc -eq 0 ] || exit 1
O=gpurun_out/r6n.txt; : > $O
SH="65536,768,3072,nt, 65536,768,768,nt,--res 65536,2304,768,nt, 65536,3072,768,nt,--act=2 65536,768,3072,nn, 65536,768,768,nn, 65536,768,2304,nn, 65536,3072,768,nn,--act=4"
for rnd in 1 2; do for band in 1 0; do for s in $SH; do
  IFS=, read M N K L X <<< "$s"
  REPLICANN_GEMM_BAND=$band timeout -k 10 60 python3 scripts/gemm_one.py $M $N $K $L --cfg 9 --iters 30 ${X/=/ } 2>/dev/null | sed "s/^/band=$band /" >> $O || exit 1
done; done; done
for rnd in 1 2; do for band in 1 0; do
  REPLICANN_GEMM_BAND=$band timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('band=$band bench', d['value'], d['ms_per_step'])" >> $O || exit 1
done; done
cat $O
