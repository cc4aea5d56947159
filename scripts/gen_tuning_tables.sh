#!/bin/bash
# Regenerate the committed GEMM tuning tables (replicann_amd/tuning/gemm_<model>.json) on a GPU box:
# each BASELINE model's bench step runs with table loading disabled, so the runtime autotuner
# measures every shape, and bench.py writes the measured table to gpurun_out/gemm_tuning_<model>.json.
# Copy those files into replicann_amd/tuning/ afterwards (scripts/install_tuning_tables.py).
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for m in gpt2-small gpt2-medium gpt2-medium-fp8 vit-b16 resnet18; do
  REPLICANN_GEMM_TABLES=0 timeout -k 10 400 python bench.py --model $m --steps 3 --warmup 2 \
    > gpurun_out/tune_$m.log 2>&1 || { echo "tuning run $m failed"; tail -5 gpurun_out/tune_$m.log; exit 1; }
  echo "$m: $(grep '^{' gpurun_out/tune_$m.log | cut -c1-200)"
done
