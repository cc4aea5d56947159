#!/bin/bash
# round 6 call AC: 8-wave (256-query) streaming causal forward vs HEAD's 4-wave one (ab/_C_h.so), alternating on one
# box: numerics, attention timing + memory-side reads, GPT-2-small step
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/pmc_mem2; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py -k "attention or attn" > gpurun_out/r6ac_tests.log 2>&1; rc=$?
tail -1 gpurun_out/r6ac_tests.log; [ $rc -eq 0 ] || exit 1
for i in 1 2; do
REPLICANN_SO=$PWD/ab/_C_h.so timeout -k 10 200 python3 scripts/attn_ab.py 64 --rounds 4 > gpurun_out/r6ac_ah$i.log 2>&1 || exit 1
timeout -k 10 200 python3 scripts/attn_ab.py 64 --rounds 4 > gpurun_out/r6ac_an$i.log 2>&1 || exit 1
echo "h$i $(grep attn_fwd gpurun_out/r6ac_ah$i.log | grep -o '"ms": [0-9.]*')  n$i $(grep attn_fwd gpurun_out/r6ac_an$i.log | grep -o '"ms": [0-9.]*')"
done
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d gpurun_out/pmc_mem2 -o n -- python3 scripts/attn_ab.py 64 --rounds 1 > /dev/null 2>&1 && \
python3 scripts/pmc_summary.py gpurun_out/pmc_mem2/n_counter_collection.csv --match attn_fwd > gpurun_out/r6ac_pmc.txt 2>&1 || exit 1
cut -c1-300 gpurun_out/r6ac_pmc.txt
for i in 1 2; do
REPLICANN_SO=$PWD/ab/_C_h.so timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r6ac_h$i.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r6ac_n$i.log 2>&1 || exit 1
echo "gpt2s h$i $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r6ac_h$i.log)  n$i $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r6ac_n$i.log)"
done
