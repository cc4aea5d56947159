#!/bin/bash
# Run GPU steps in order; each under its own timeout.  Test FAILURES (exit 1)
# do not stop the sequence; a crash/abort/timeout (>=124, signals) does.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # run <name> <timeout_s> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/steps.log
  local t0=$(date +%s)
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc ($(( $(date +%s) - t0 ))s)" | tee -a gpurun_out/steps.log
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ge 124 ] || [ $rc -lt 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return 0
}
for step in "$@"; do
  case $step in
    ops) run ops 900 python -m pytest tests/test_ops_gpu.py -x -q ;;
    opsk) run opsk 900 python -m pytest tests/test_ops_gpu.py -q ;;
    models) run models 600 python -m pytest tests/test_models.py -m gpu -q ;;
    gpu_all) run gpu_all 1200 python -m pytest tests -m gpu -q ;;
    conv) run conv 900 python -m pytest tests/test_convergence_gpu.py -q ;;
    traj) run traj 900 python scripts/check_trajectory.py --model gpt2-small gpt2-medium vit-b16 resnet18 --steps 8 ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 600 python bench.py --steps 10 --warmup 3 ;;
    bench_small) run bench_small 600 python bench.py --steps 5 --warmup 2 --batch 4 ;;
    bench_configs) run bench_med 600 python bench.py --model gpt2-medium --steps 5 --warmup 2 && run bench_med_fp8 600 python bench.py --model gpt2-medium-fp8 --steps 5 --warmup 2 && run bench_vit 600 python bench.py --model vit-b16 --steps 5 --warmup 2 && run bench_resnet 600 python bench.py --model resnet18 --steps 5 --warmup 2 ;;
    prof) run prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 3 --warmup 2 ;;
    bench_eager) run bench_eager 600 python bench.py --steps 10 --warmup 3 --graph off ;;
    tprof) run tprof 600 python bench.py --steps 3 --warmup 2 --profile-steps 2 ;;
    microbench) run microbench 600 python scripts/microbench.py ;;
    mbgemm) run mbgemm 600 python scripts/microbench.py gemm ;;
    mbattn) run mbattn 300 python scripts/microbench.py attn ln xent ;;
    det) run det 300 python -m pytest tests/test_determinism_gpu.py -q ;;
    stock) run stock 600 python scripts/bench_stock_torch.py --steps 10 --warmup 3 ;;
    stock_all) for m in gpt2-small gpt2-medium vit-b16 resnet18; do run stock_$m 600 python scripts/bench_stock_torch.py --model $m --steps 5 --warmup 2; done ;;
    *) ncustom=$(( ${ncustom:-0} + 1 )); run custom$ncustom 600 bash -c "$step" ;;
  esac
done
