#!/bin/bash
# round 6 call AI: same-box A/B of the dQ-bias reduce-scatter: (h) HEAD (LDS reduction, ab/_C_h.so) vs (n) tree, attention
# backward with / without bias partials and the ViT-B/16 step
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for i in 1 2; do
for v in h n; do
  if [ $v = h ]; then export REPLICANN_SO=$PWD/ab/_C_h.so; else unset REPLICANN_SO; fi
  timeout -k 10 200 python3 scripts/attn_ab.py 512 --T 197 --noncausal --rounds 4 > gpurun_out/r6ai_${v}p$i.log 2>&1 || exit 1
  timeout -k 10 200 python3 scripts/attn_ab.py 512 --T 197 --noncausal --rounds 4 --bias-grad > gpurun_out/r6ai_${v}b$i.log 2>&1 || exit 1
  echo "$v$i plain $(grep attn_bwd gpurun_out/r6ai_${v}p$i.log | grep -o '"ms": [0-9.]*')  bias $(grep attn_bwd gpurun_out/r6ai_${v}b$i.log | grep -o '"ms": [0-9.]*')"
done; done
for i in 1 2; do
REPLICANN_SO=$PWD/ab/_C_h.so timeout -k 10 300 python -u bench.py --model vit-b16 --steps 10 --warmup 3 > gpurun_out/r6ai_vh$i.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --model vit-b16 --steps 10 --warmup 3 > gpurun_out/r6ai_vn$i.log 2>&1 || exit 1
echo "vit h$i $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r6ai_vh$i.log)  n$i $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r6ai_vn$i.log)"
done
