"""Per-step kernel time breakdown of a training run's last complete steps, from a rocprofv3
kernel trace (``--kernel-trace --output-format csv``: ``*_kernel_trace.csv``) or a rocpd sqlite
database (``*_results.db``).

Steps are the intervals between consecutive launches of a MARKER kernel that runs exactly once
per step (default: the fused optimizer, ``adamw_k`` / ``sgd_k``).  Only COMPLETE intervals are
counted — [marker i, marker i+1) for the last ``--steps`` pairs — so a kernel is never split
across a boundary or counted for a partial step, and the per-step kernel sum can be checked
against the interval length (the "span"): on a saturated GPU they agree within launch gaps.

    python scripts/prof_steps.py gpurun_out/prof/run_kernel_trace.csv --steps 3 [--marker sgd_k] [--top 30]
"""
import argparse
import csv
import sqlite3
from collections import defaultdict


def load(path):
    """[(name, start_ns, end_ns)] sorted by start."""
    if path.endswith(".csv"):
        with open(path) as f:
            rows = [(r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in csv.DictReader(f)]
    else:
        con = sqlite3.connect(path)
        rows = con.execute("select name, start, end from kernels").fetchall()
    return sorted(rows, key=lambda r: r[1])


def breakdown(rows, steps, markers):
    marks = [r[1] for r in rows if any(m in r[0] for m in markers)]
    if len(marks) < steps + 1:
        raise SystemExit(f"only {len(marks)} marker launches ({markers}): need steps + 1 = {steps + 1}")
    lo, hi = marks[-steps - 1], marks[-1]
    sel = [r for r in rows if lo <= r[1] < hi]
    agg = defaultdict(lambda: [0, 0.0])
    for n, s, e in sel:
        agg[n][0] += 1
        agg[n][1] += (e - s) / 1e6
    busy = sum(v[1] for v in agg.values()) / steps
    span = (hi - lo) / 1e6 / steps
    return agg, busy, span, len(sel) / steps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--marker", action="append", default=None,
                    help="substring of the once-per-step kernel (repeatable; default adamw_k, sgd_k)")
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args()
    markers = a.marker or ["adamw_k", "sgd_k"]
    agg, busy, span, launches = breakdown(load(a.trace), a.steps, markers)
    print(f"steps={a.steps}  wall/step={span:.3f} ms  kernel-busy/step={busy:.3f} ms  launches/step={launches:.0f}")
    print(" ms/step     % n/step  kernel")
    for n, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[: a.top]:
        print(f"{t / a.steps:8.3f} {100 * t / a.steps / busy:5.1f} {c / a.steps:6.0f}  {n[:110]}")


if __name__ == "__main__":
    main()
