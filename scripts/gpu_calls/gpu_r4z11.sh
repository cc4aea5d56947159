#!/bin/bash
# round 4 (call Z11): kernel breakdowns of the GPT-2-medium bf16 and fp8 (forward GEMMs) steps at HEAD, for the
# fp8 item's next round (what the quantisation and the K = 1024 GEMMs cost per step).
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for m in gpt2-medium gpt2-medium-fp8; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_z11_$m -o run -- python3 bench.py --model $m --steps 3 --warmup 2 > gpurun_out/z11_$m.log 2>&1 || { echo "prof $m failed"; tail -3 gpurun_out/z11_$m.log; exit 1; }
  python scripts/prof_steps.py gpurun_out/prof_z11_$m/run_kernel_trace.csv --steps 3 > gpurun_out/z11_${m}_steps.txt 2>&1
  echo "=== $m $(grep -o '"value": [0-9.]*' gpurun_out/z11_$m.log)"; head -26 gpurun_out/z11_${m}_steps.txt | cut -c1-150
done
exit 0
