#!/bin/bash
# round 6 call Z: ViT-B/16 bench alternating on one box: (h) HEAD build ab/_C_h.so vs (n) tree (dV bias partials on the MFMA)
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for i in 1 2; do
REPLICANN_SO=$PWD/ab/_C_h.so timeout -k 10 300 python -u bench.py --model vit-b16 --steps 10 --warmup 3 > gpurun_out/r6z_h$i.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --model vit-b16 --steps 10 --warmup 3 > gpurun_out/r6z_n$i.log 2>&1 || exit 1
echo "h$i $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r6z_h$i.log)  n$i $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r6z_n$i.log)"
done
