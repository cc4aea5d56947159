#!/bin/bash
# round 5 (call E): GPT-2-small bench, this tree vs the round-4 tree (_r4/, built in-tree from commit 3bafd8f),
# alternating; kernel breakdowns of both; GPT-2-medium-fp8 breakdown (which fp8 kernels run); PMC counter list.
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
R=$PWD
for r in 1 2; do
  (cd $R/_r4 && timeout -k 10 200 python bench.py > $R/gpurun_out/r5e_old_$r.log 2>&1) || { echo "old bench failed"; tail -3 gpurun_out/r5e_old_$r.log; exit 1; }
  echo "old r$r: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5e_old_$r.log)"
  timeout -k 10 200 python bench.py > gpurun_out/r5e_new_$r.log 2>&1 || { echo "new bench failed"; tail -3 gpurun_out/r5e_new_$r.log; exit 1; }
  echo "new r$r: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5e_new_$r.log)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_5e_new -o run -- python3 bench.py --steps 3 --warmup 2 > gpurun_out/r5e_prof_new.log 2>&1 || { echo "prof new failed"; exit 1; }
python scripts/prof_steps.py gpurun_out/prof_5e_new/run_kernel_trace.csv --steps 3 > gpurun_out/r5e_steps_new.txt 2>&1
(cd _r4 && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_5e_old -o run -- python3 bench.py --steps 3 --warmup 2 > $R/gpurun_out/r5e_prof_old.log 2>&1) || { echo "prof old failed"; exit 1; }
python scripts/prof_steps.py gpurun_out/prof_5e_old/run_kernel_trace.csv --steps 3 > gpurun_out/r5e_steps_old.txt 2>&1
head -16 gpurun_out/r5e_steps_new.txt | cut -c1-150; head -16 gpurun_out/r5e_steps_old.txt | cut -c1-150
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_5e_m8 -o run -- python3 bench.py --model gpt2-medium-fp8 --steps 3 --warmup 2 > gpurun_out/r5e_prof_m8.log 2>&1 || { echo "prof m8 failed"; exit 1; }
python scripts/prof_steps.py gpurun_out/prof_5e_m8/run_kernel_trace.csv --steps 3 > gpurun_out/r5e_steps_m8.txt 2>&1
head -30 gpurun_out/r5e_steps_m8.txt | cut -c1-150
rm -rf gpurun_out/prof_5e_new gpurun_out/prof_5e_old gpurun_out/prof_5e_m8
timeout -k 10 60 rocprofv3 -L > gpurun_out/r5e_counters.txt 2>&1; echo "counters rc=$?"
