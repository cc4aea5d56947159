#!/bin/bash
# round 6 call H: fp8 numerics against a bf16 seed-to-seed noise floor (200 steps, GPT-2-medium, b16)
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python3 -u scripts/fp8_noise_floor.py 200 16 1e-4 > gpurun_out/r6h_noise.jsonl 2> gpurun_out/r6h_noise.err || { echo "noise floor failed"; tail -5 gpurun_out/r6h_noise.err; exit 1; }
grep -v '"run"' gpurun_out/r6h_noise.jsonl
