#!/bin/bash
# round 3: saved-activation L2 prefetch in act-backward epilogues — correctness, then A/B vs no prefetch
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "act_backward or gelu_saved or persistent_multi_tile or mlp_fused" > gpurun_out/pf_test.log 2>&1
rc=$?; tail -3 gpurun_out/pf_test.log; [ $rc -eq 0 ] || exit 1
for v in dev dev_pf dev; do
  REPLICANN_SO=$PWD/ab/${v}_C.so timeout -k 10 300 python scripts/gemm_msweep.py --shapes fc1_dgrad_act6,proj_fwd --m 65536,131072 \
    > gpurun_out/pf_$v.jsonl 2> gpurun_out/pf_$v.err || { tail -20 gpurun_out/pf_$v.err; exit 1; }
  echo "== $v"; cat gpurun_out/pf_$v.jsonl
done
