#!/bin/bash
# round 4 (call I): persistent-GEMM start stagger (REPLICANN_GEMM_STAGGER) — do the K = 768 shapes'
# epilogue bursts, synchronised across all 256 CUs, cost the ~10 us per tile the PMC suggests?
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for r in 1 2; do
  for sg in 0 1 2 3; do
    REPLICANN_GEMM_STAGGER=$sg timeout -k 10 200 python scripts/gemm_msweep.py --m 65536 --rounds 2 \
      --shapes proj_fwd,qkv_fwd,fc1_fwd,fc1_dgrad_act6,fc2_fwd > gpurun_out/stagger_${sg}_$r.log 2>&1 || { echo "sweep $sg failed"; exit 1; }
    echo "stagger=$sg r$r: $(grep '"shape"' gpurun_out/stagger_${sg}_$r.log | python -c "
import sys,json,collections
d=collections.defaultdict(list)
for l in sys.stdin: r=json.loads(l); d[r['shape']].append(r['us'])
print(' '.join('%s=%.1f' % (k, min(v)) for k, v in d.items()))")"
  done
done
for r in 1 2; do
  for sg in 0 2; do
    REPLICANN_GEMM_STAGGER=$sg timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/stagger_bench_${sg}_$r.log 2>&1 || { echo "bench failed"; exit 1; }
    echo "bench stagger=$sg r$r: $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/stagger_bench_${sg}_$r.log | tr '\n' ' ')"
  done
done
exit 0
