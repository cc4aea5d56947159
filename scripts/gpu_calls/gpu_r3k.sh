#!/bin/bash
# round 3: what the epilogue's full-tile operand read (residual / saved gelu') costs: default vs no-aux ablation
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in dev dev_noaux; do
  REPLICANN_SO=$PWD/ab/${v}_C.so timeout -k 10 300 python scripts/gemm_msweep.py --shapes proj_fwd,fc2_fwd,fc1_dgrad_act6,qkv_fwd --m 65536 \
    > gpurun_out/aux_$v.jsonl 2> gpurun_out/aux_$v.err || { tail -20 gpurun_out/aux_$v.err; exit 1; }
  echo "== $v"; cat gpurun_out/aux_$v.jsonl
done
