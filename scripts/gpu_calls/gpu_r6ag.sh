#!/bin/bash
# round 6 call AG: cost of the QKV bias partials in the resident backward (ViT shape), with / without, alternating
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for i in 1 2; do
timeout -k 10 200 python3 scripts/attn_ab.py 512 --T 197 --noncausal --rounds 4 > gpurun_out/r6ag_n$i.log 2>&1 || exit 1
timeout -k 10 200 python3 scripts/attn_ab.py 512 --T 197 --noncausal --rounds 4 --bias-grad > gpurun_out/r6ag_b$i.log 2>&1 || { tail -5 gpurun_out/r6ag_b$i.log; exit 1; }
echo "plain$i $(grep attn_bwd gpurun_out/r6ag_n$i.log | grep -o '"ms": [0-9.]*')  bias$i $(grep attn_bwd gpurun_out/r6ag_b$i.log | grep -o '"ms": [0-9.]*')"
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r6ag_prof -o run -- python3 scripts/attn_ab.py 512 --T 197 --noncausal --rounds 1 --bias-grad > /dev/null 2>&1 || exit 1
find gpurun_out/r6ag_prof -name "*kernel_stats.csv" | head -1 | xargs -I{} sh -c 'cut -d, -f1-4 {} | head -8'
