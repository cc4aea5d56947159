#!/bin/bash
# round 6 call I: bf16 cfg 11 (one wave per SIMD, now with the XCD-banded walk) vs cfg 9 on the GPT-2-small plain shapes
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/r6i.txt; : > $O
SH="65536,2304,768,nt, 65536,768,768,nt,--res 65536,768,3072,nt,--res 65536,50304,768,nt, 65536,768,3072,nn, 65536,768,768,nn, 65536,768,2304,nn, 65536,768,50304,nn,"
for rnd in 1 2; do for cfg in 9 11; do for s in $SH; do
  IFS=, read M N K L X <<< "$s"
  timeout -k 10 60 python3 scripts/gemm_one.py $M $N $K $L --cfg $cfg --iters 30 $X 2>/dev/null | sed "s/^/cfg=$cfg /" >> $O || exit 1
done; done; done
cat $O
