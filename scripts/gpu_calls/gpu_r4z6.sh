#!/bin/bash
# round 4 (call Z6): committed GEMM table A/B for GPT-2-small's attention c_proj forward (65536x768x768 +
# residual): the committed pick (cfg 1, one tile per block) vs the persistent kernel (cfg 9), which the
# round-4 sweep measured 3-15 % faster in isolation (profiles/gemm_staged_ab_r4f.txt).  Alternating runs.
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=replicann_amd/tuning/gemm_gpt2-small.json
cp $T gpurun_out/z6_table_committed.json
python - <<'PY'
import json
t = json.load(open("replicann_amd/tuning/gemm_gpt2-small.json"))
for e in t:
    if (e["M"], e["N"], e["K"], e["ta"], e["tb"], e["epi"]) == (65536, 768, 768, 0, 1, 3):
        e["cfg"] = 9
json.dump(t, open("gpurun_out/z6_table_cfg9.json", "w"))
PY
for r in 1 2 3; do
  cp gpurun_out/z6_table_committed.json $T
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/z6_a$r.log 2>&1 || { echo "bench a failed"; exit 1; }
  echo "committed r$r: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/z6_a$r.log)"
  cp gpurun_out/z6_table_cfg9.json $T
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/z6_b$r.log 2>&1 || { echo "bench b failed"; exit 1; }
  echo "proj_fwd cfg9 r$r: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/z6_b$r.log)"
done
cp gpurun_out/z6_table_committed.json $T
exit 0
