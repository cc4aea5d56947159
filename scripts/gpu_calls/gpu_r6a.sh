#!/bin/bash
# round 6 baseline: headline bench, attention kernel timings (GPT-2-small causal, ViT T=197), GPT-2-small breakdown
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 240 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r6a_bench.log 2>&1 || { echo bench failed; exit 1; }
tail -1 gpurun_out/r6a_bench.log
timeout -k 10 120 python3 scripts/attn_ab.py 64 --rounds 3 > gpurun_out/r6a_attn.log 2>&1 || { echo attn failed; exit 1; }
timeout -k 10 120 python3 scripts/attn_ab.py 512 --rounds 3 --T 197 --noncausal >> gpurun_out/r6a_attn.log 2>&1 || { echo attn197 failed; exit 1; }
cat gpurun_out/r6a_attn.log
M=gpt2-small
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_brk_$M -o run -- python3 bench.py --model $M --steps 3 --warmup 2 > gpurun_out/r6a_brk_$M.log 2>&1 || { echo "prof $M failed"; exit 1; }
python scripts/prof_steps.py gpurun_out/prof_brk_$M/run_kernel_trace.csv --steps 3 > gpurun_out/r6a_steps_$M.txt 2>&1
rm -rf gpurun_out/prof_brk_$M
head -40 gpurun_out/r6a_steps_$M.txt | cut -c1-160
