#!/bin/bash
# round 4 (call G): fp8 backward for GPT-2-medium — step A/B (bf16 model, fp8 forward only, + fp8 weight
# gradients, + fp8 data gradients), per-shape backward GEMM A/B, 50-step fp8-vs-bf16 trajectory with
# the fp8 backward on; PMC of the staged vs unstaged GEMM epilogues.
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
step() {  # step <name> <timeout> cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/$n.log 2>&1; local rc=$?
  echo "=== $n rc=$rc $(grep -v amdgpu.ids gpurun_out/$n.log | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|max_rel[a-z_]*": [0-9.e-]*' | tr '\n' ' ')"
  return $rc
}
for r in 1 2; do
  step m_bf16_$r 300 python bench.py --model gpt2-medium --steps 6 --warmup 3 || exit 1
  step m8_fwd_$r 300 python bench.py --model gpt2-medium-fp8 --steps 6 --warmup 3 || exit 1
  REPLICANN_FP8_WGRAD=1 step m8_w_$r 300 python bench.py --model gpt2-medium-fp8 --steps 6 --warmup 3 || exit 1
  REPLICANN_FP8_WGRAD=1 REPLICANN_FP8_DGRAD=1 step m8_wd_$r 300 python bench.py --model gpt2-medium-fp8 --steps 6 --warmup 3 || exit 1
done
step fp8_bwd_ab 300 python scripts/fp8_bwd_ab.py 16384 3 || exit 1
grep -v amdgpu.ids gpurun_out/fp8_bwd_ab.log | grep "{" | head -20
REPLICANN_FP8_WGRAD=1 REPLICANN_FP8_DGRAD=1 step traj_m8 600 python scripts/fp8_trajectory.py 50 16 1e-4 || exit 1
grep -v amdgpu.ids gpurun_out/traj_m8.log | tail -2
step pmc_staged 600 bash scripts/pmc_staged.sh || exit 1
python scripts/pmc_summary.py gpurun_out/pmc_stg/*_counter_collection.csv --match gemm_pk > gpurun_out/pmc_staged_summary.txt 2>&1
head -40 gpurun_out/pmc_staged_summary.txt
exit 0
