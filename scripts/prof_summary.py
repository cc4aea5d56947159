"""Per-step kernel breakdown from a rocprofv3 ``--kernel-trace`` CSV.

Steps are delimited by the optimizer kernel (one ``adamw``/``sgd`` launch per
step); the last ``--steps`` complete steps are averaged so warm-up, autotuning
and graph capture are excluded.

    python scripts/prof_summary.py gpurun_out/prof/run_kernel_trace.csv --steps 3
"""

import argparse
import csv
import re
import subprocess
from collections import defaultdict


def demangle(names):
    names = list(names)
    try:
        out = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True, check=True)
        return dict(zip(names, out.stdout.split("\n")))
    except Exception:
        return {n: n for n in names}


def short(name):
    n = name.replace("(anonymous namespace)::", "").replace("rn_gemm_detail::", "")
    n = re.sub(r"^void ", "", n)
    n = re.sub(r"\(.*$", "", n)
    return n[:100]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--marker", default="adamw|sgd_k|sgd_step")
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    rows = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    dm = demangle({n for _, _, n in rows})
    rows = sorted((s, e, dm.get(n, n)) for s, e, n in rows)
    mk = re.compile(a.marker)
    ends = [i for i, (_, _, n) in enumerate(rows) if mk.search(n)]
    if len(ends) < a.steps + 1:
        raise SystemExit(f"only {len(ends)} optimizer launches found")
    lo, hi = ends[-a.steps - 1] + 1, ends[-1] + 1
    sel = rows[lo:hi]
    wall = (sel[-1][1] - sel[0][0]) / 1e6 / a.steps
    agg = defaultdict(lambda: [0, 0.0])
    for s, e, n in sel:
        k = short(n)
        agg[k][0] += 1
        agg[k][1] += (e - s) / 1e6
    busy = sum(v[1] for v in agg.values()) / a.steps
    print(f"steps={a.steps}  wall/step={wall:.3f} ms  kernel-busy/step={busy:.3f} ms  "
          f"launches/step={len(sel) / a.steps:.0f}")
    print(f"{'ms/step':>8} {'%':>5} {'n/step':>6}  kernel")
    for k, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:a.top]:
        print(f"{t / a.steps:8.3f} {100 * t / a.steps / busy:5.1f} {c / a.steps:6.0f}  {k}")


if __name__ == "__main__":
    main()
