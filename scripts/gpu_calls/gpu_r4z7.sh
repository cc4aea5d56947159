#!/bin/bash
# round 4 (call Z7): committed GEMM table A/B for GPT-2-small's attention c_proj weight gradient (768x768,
# K = 65,536 tokens): committed cfg 8 (256x128 tiles) split 14 vs the persistent cfg 9 at split 14 / 28.
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=replicann_amd/tuning/gemm_gpt2-small.json
cp $T gpurun_out/z7_a.json
python - <<'PY'
import json
for tag, cfg, sp in (("b", 9, 14), ("c", 9, 28)):
    t = json.load(open("replicann_amd/tuning/gemm_gpt2-small.json"))
    for e in t:
        if (e["M"], e["N"], e["K"], e["ta"], e["tb"]) == (768, 768, 65536, 1, 0):
            e["cfg"], e["split"] = cfg, sp
    json.dump(t, open(f"gpurun_out/z7_{tag}.json", "w"))
PY
for r in 1 2 3; do
  for v in a b c; do
    cp gpurun_out/z7_$v.json $T
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/z7_$v$r.log 2>&1 || { echo "bench $v failed"; tail -3 gpurun_out/z7_$v$r.log; cp gpurun_out/z7_a.json $T; exit 1; }
    echo "$v r$r: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/z7_$v$r.log)"
  done
done
cp gpurun_out/z7_a.json $T
exit 0
