#!/bin/bash
# round 5 (call R): ResNet-18 / ViT-B/16 benches on this tree, per-shape conv weight-gradient rates, ResNet step breakdown.
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for M in resnet18 vit-b16; do
  timeout -k 10 300 python -u bench.py --model $M --steps 10 --warmup 3 > gpurun_out/r5r_$M.log 2>&1 || { echo "bench $M failed"; tail -5 gpurun_out/r5r_$M.log; exit 1; }
  echo "$M: $(grep -o '"value": [0-9.]*' gpurun_out/r5r_$M.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5r_$M.log)"
done
timeout -k 10 200 python -u scripts/conv_ab.py > gpurun_out/r5r_conv_ab.log 2>&1 || { echo "conv_ab failed"; tail -5 gpurun_out/r5r_conv_ab.log; exit 1; }
cat gpurun_out/r5r_conv_ab.log
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_5r -o run -- python3 bench.py --model resnet18 --steps 5 --warmup 2 > gpurun_out/r5r_prof.log 2>&1 || { echo "prof failed"; exit 1; }
python scripts/prof_steps.py gpurun_out/prof_5r/run_kernel_trace.csv --steps 5 > gpurun_out/r5r_steps_resnet.txt 2>&1
cp gpurun_out/prof_5r/run_kernel_trace.csv gpurun_out/r5r_resnet_trace.csv 2>/dev/null
rm -rf gpurun_out/prof_5r
head -24 gpurun_out/r5r_steps_resnet.txt | cut -c1-150
