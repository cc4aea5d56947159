"""Per-step kernel time breakdown from a rocprofv3 --kernel-trace sqlite (rocpd) database, counting only the
LAST `--steps` training steps (autotuner sweeps and warm-up excluded).  A step boundary is every
`--per-step`-th launch of the marker kernel (default: the attention forward, once per layer).

    python scripts/prof_steps.py gpurun_out/prof/x_results.db --steps 5 --per-step 12 [--top 30]
"""
import argparse
import sqlite3
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--per-step", type=int, required=True, help="marker launches per step (n_layer)")
    ap.add_argument("--marker", default="attn_fwd")
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args()
    con = sqlite3.connect(a.db)
    rows = con.execute("select name, start, end from kernels order by start").fetchall()
    marks = [r[1] for r in rows if a.marker in r[0]]
    cut = marks[-a.steps * a.per_step]
    sel = [r for r in rows if r[1] >= cut]
    agg = defaultdict(lambda: [0, 0.0])
    for n, s, e in sel:
        agg[n][0] += 1
        agg[n][1] += (e - s) / 1e6
    tot = sum(v[1] for v in agg.values())
    span = (sel[-1][2] - sel[0][1]) / 1e6
    print(f"# last {a.steps} steps: kernel time {tot / a.steps:.2f} ms/step, span {span / a.steps:.2f} ms/step")
    for n, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[: a.top]:
        print(f"{t / a.steps:8.3f} ms/step {c // a.steps:5d}x  {n[:120]}")


if __name__ == "__main__":
    main()
