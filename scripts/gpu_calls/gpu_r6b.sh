#!/bin/bash
# round 6 call B: XCD-banded persistent-GEMM walk (REPLICANN_GEMM_BAND) A/B — per-shape timings, memory-side
# reads (PMC), GPT-2-small step alternating
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/r6b.txt; : > $O
SH="65536,2304,768,nt 65536,768,768,nt 65536,3072,768,nt 65536,768,3072,nt 65536,768,3072,nn 65536,768,768,nn 65536,768,2304,nn 65536,50304,768,nt"
for rnd in 1 2; do for band in 1 0; do for s in $SH; do
  IFS=, read M N K L <<< "$s"
  REPLICANN_GEMM_BAND=$band timeout -k 10 60 python3 scripts/gemm_one.py $M $N $K $L --cfg 9 --iters 30 2>/dev/null | sed "s/^/band=$band /" >> $O || exit 1
done; done; done
for band in 1 0; do
  REPLICANN_GEMM_BAND=$band timeout -k 10 60 python3 scripts/gemm_one.py 65536 3072 1024 nt --fp8 11 --iters 30 2>/dev/null | sed "s/^/band=$band fp8 /" >> $O || exit 1
  REPLICANN_GEMM_BAND=$band timeout -k 10 60 python3 scripts/gemm_one.py 65536 1024 4096 nt --fp8 11 --iters 30 2>/dev/null | sed "s/^/band=$band fp8 /" >> $O || exit 1
done
for band in 1 0; do
  REPLICANN_GEMM_BAND=$band timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/pmc_band -o b${band}_fc2 -- python3 scripts/gemm_one.py 65536 768 3072 nt --cfg 9 --iters 5 > /dev/null 2>&1 || exit 1
  REPLICANN_GEMM_BAND=$band timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/pmc_band -o b${band}_qkv -- python3 scripts/gemm_one.py 65536 2304 768 nt --cfg 9 --iters 5 > /dev/null 2>&1 || exit 1
done
for f in gpurun_out/pmc_band/*_counter_collection.csv; do echo "== $f" >> $O; python3 scripts/pmc_summary.py $f --match gemm >> $O 2>&1; done
for rnd in 1 2; do for band in 1 0; do
  REPLICANN_GEMM_BAND=$band timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('band=$band bench', d['value'], d['ms_per_step'])" >> $O || exit 1
done; done
cat $O
