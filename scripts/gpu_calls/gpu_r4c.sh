#!/bin/bash
# round 4 (call B2): plain vs comm-proxy graph / eager GPT-2-small rows (verdict r3 item 2), attention
# PMC, ViT-B/16 step profile, numerics records at HEAD (item 5), fp8 weight-gradient A/B
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
step() {  # step <name> <timeout> cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/$n.log 2>&1; local rc=$?
  echo "=== $n rc=$rc"; grep -v "amdgpu.ids" gpurun_out/$n.log | grep -o '"ms_per_step": [0-9.]*' | tail -1; grep -E "max_rel" gpurun_out/$n.log | tail -1
  return $rc
}
for r in 1 2; do
  step plain_eager_$r 300 python bench.py --steps 10 --warmup 3 --graph off || exit 1
  step proxy_graph_$r 300 python bench.py --steps 10 --warmup 3 --ddp on --comm proxy || exit 1
  step proxy_eager_$r 300 python bench.py --steps 10 --warmup 3 --ddp on --comm proxy --graph off || exit 1
done
step pmc_attn 400 bash scripts/pmc_attn.sh "64 --rounds 1" attn4 || exit 1
python scripts/pmc_summary.py gpurun_out/pmc_attn/attn4*_counter_collection.csv --match attn > gpurun_out/pmc_attn_summary.txt 2>&1
step prof_vit 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_4c_vit -o run -- python3 bench.py --model vit-b16 --steps 3 --warmup 2 || exit 1
python scripts/prof_steps.py gpurun_out/prof_4c_vit/run_kernel_trace.csv --steps 3 > gpurun_out/prof_4c_vit_steps.txt 2>&1
step traj_s 600 python scripts/check_trajectory.py --model gpt2-small --steps 100 --lr 1e-4 --batch 16 --threshold 0.02
exit 0
