#!/bin/bash
# round 6 call M: what limits the bf16 GEMM (verdict r5 item 2) — per-CU vs shared resource: the persistent
# kernel on fewer CUs (REPLICANN_GEMM_RESERVE leaves CUs idle), s_fc2 / s_qkv / LM head; then the counter list
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/r6m.txt; : > $O
for rnd in 1 2; do for res in 0 64 128; do for s in 65536,768,3072 65536,2304,768 65536,50304,768; do
  IFS=, read M N K <<< "$s"
  timeout -k 10 60 python3 scripts/gemm_one.py $M $N $K nt --cfg 9 --iters 20 --reserve $res 2>/dev/null | sed "s/^/reserve=$res cus=$((256-res)) /" >> $O || exit 1
done; done; done
cat $O
timeout -k 5 60 rocprofv3 -L > gpurun_out/r6m_counters.txt 2>&1 || true
grep -o "TA_[A-Z_]*\|TCP_[A-Z_]*\|TD_[A-Z_]*" gpurun_out/r6m_counters.txt | sort -u | head -80 > gpurun_out/r6m_ta_tcp.txt
wc -l gpurun_out/r6m_ta_tcp.txt
