#!/bin/bash
# round 6 call R: ViT-B/16 bench with the resident attention kernels; PMC on the resident fwd / bwd
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --model vit-b16 --steps 10 --warmup 3 > gpurun_out/r6r_vit.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r6r_vit.log; exit 1; }
echo "vit: $(grep -o '"value": [0-9.]*' gpurun_out/r6r_vit.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r6r_vit.log)"
timeout -k 10 200 bash scripts/pmc_attn.sh "512 --T 197 --noncausal --rounds 1" vitres && \
python3 scripts/pmc_summary.py gpurun_out/pmc_attn/vitres*_counter_collection.csv --match attn > gpurun_out/r6r_pmc.txt 2>&1; rc=$?
cat gpurun_out/r6r_pmc.txt | cut -c1-400; exit $rc
