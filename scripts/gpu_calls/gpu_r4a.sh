#!/bin/bash
# round 4: GPU tests after the knob/variant cleanup and the staged GEMM epilogue; staged vs unstaged
# A/B (GEMM sweep + GPT-2-small step); plain vs comm-proxy (graph / eager) rows (verdict r3 item 2);
# numerics records at HEAD (item 5)
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
step() {  # step <name> <timeout> cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/$n.log 2>&1; local rc=$?
  echo "=== $n rc=$rc"; grep -v "amdgpu.ids" gpurun_out/$n.log | grep -o '"ms_per_step": [0-9.]*' | tail -1; grep -E "passed|failed|smoke ok|max_rel" gpurun_out/$n.log | tail -1
  return $rc
}
step tr8_probe 30 ./scripts/dev/tr8_probe || exit 1
step t_staged 300 python -u -m pytest tests/test_gemm_staged_gpu.py tests/test_reference_parity_gpu.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider || exit 1
step gpu_all 1000 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider || exit 1
step smoke 200 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
step msweep 300 python scripts/gemm_msweep.py --m 65536 --staged 0,1 --rounds 3 --shapes proj_fwd,fc2_fwd,fc1_dgrad_act6,qkv_fwd || exit 1
for r in 1 2; do
  step plain_$r 300 python bench.py --steps 10 --warmup 3 || exit 1
  REPLICANN_GEMM_STAGED=0 step unstaged_$r 300 python bench.py --steps 10 --warmup 3 || exit 1
done
for r in 1 2; do
  step plain_eager_$r 300 python bench.py --steps 10 --warmup 3 --graph off || exit 1
  step proxy_graph_$r 300 python bench.py --steps 10 --warmup 3 --ddp on --comm proxy || exit 1
  step proxy_eager_$r 300 python bench.py --steps 10 --warmup 3 --ddp on --comm proxy --graph off || exit 1
done
step prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_4a -o run -- python3 bench.py --steps 3 --warmup 2 || exit 1
python scripts/prof_steps.py gpurun_out/prof_4a/run_kernel_trace.csv --steps 3 > gpurun_out/prof_4a_steps.txt 2>&1
step traj_s 600 python scripts/check_trajectory.py --model gpt2-small --steps 100 --lr 1e-4 --batch 16 --threshold 0.02
step traj_m8 600 python scripts/fp8_trajectory.py 50 16 1e-4
exit 0
