#!/bin/bash
# round 3: epilogue store cache policy (default / nt / sc0 sc1) and store ablations (DBG 32 / 64)
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
out=gpurun_out/stpol.jsonl; : > $out
run() {  # run <tag> <so> args...
  local tag=$1 so=$2; shift 2
  REPLICANN_SO=$PWD/ab/$so timeout -k 10 120 python scripts/gemm_one.py "$@" --iters 30 > gpurun_out/one.log 2>&1 || { cat gpurun_out/one.log; exit 1; }
  echo "{\"tag\": \"$tag\", \"r\": $(grep '^{' gpurun_out/one.log)}" | tee -a $out
}
for s in "65536 50304 768 nt" "65536 2304 768 nt" "65536 3072 768 nt --act 5" "65536 768 3072 nt"; do
  run default dev_C.so $s
  run nt dev_nt_C.so $s
  run sc dev_sc_C.so $s
done
for s in "65536 50304 768 nt" "65536 2304 768 nt"; do
  run dbg32_oob_stores dev_C.so $s --cfg 122
  run dbg64_no_stores dev_C.so $s --cfg 154
done
