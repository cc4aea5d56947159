#!/bin/bash
# round 4 (call H): GPT-2-small plain vs comm-proxy (graph / eager) rows — the eager form is what
# world > 1 runs (verdict r3 item 2); ViT-B/16 step profile; GPT-2-small native-vs-fp32 100-step
# trajectory (verdict r3 item 5).
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
step() {  # step <name> <timeout> cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/$n.log 2>&1; local rc=$?
  echo "=== $n rc=$rc $(grep -v amdgpu.ids gpurun_out/$n.log | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|max_rel[a-z_]*": [0-9.e-]*' | tr '\n' ' ')"
  return $rc
}
for r in 1 2; do
  step plain_graph_$r 300 python bench.py --steps 10 --warmup 3 || exit 1
  step plain_eager_$r 300 python bench.py --steps 10 --warmup 3 --graph off || exit 1
  step proxy_graph_$r 300 python bench.py --steps 10 --warmup 3 --ddp on --comm proxy || exit 1
  step proxy_eager_$r 300 python bench.py --steps 10 --warmup 3 --ddp on --comm proxy --graph off || exit 1
done
step vit 300 python bench.py --model vit-b16 --steps 8 --warmup 3 || exit 1
step prof_vit 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_4h_vit -o run -- python3 bench.py --model vit-b16 --steps 3 --warmup 2 || exit 1
python scripts/prof_steps.py gpurun_out/prof_4h_vit/run_kernel_trace.csv --steps 3 > gpurun_out/prof_4h_vit_steps.txt 2>&1
head -25 gpurun_out/prof_4h_vit_steps.txt
step traj_s 600 python scripts/check_trajectory.py --model gpt2-small --steps 100 --lr 1e-4 --batch 16 --threshold 0.02
grep -v amdgpu.ids gpurun_out/traj_s.log | tail -2 | cut -c1-400
exit 0
