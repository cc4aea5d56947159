"""rocprofv3 result analysis (N25, SURVEY.md §5 "tracing / profiling").

Two inputs, both written by ``rocprofv3 --output-format csv``:

* ``*_kernel_trace.csv`` (``--kernel-trace``): per-dispatch start/end, grid, VGPRs.
  :func:`step_breakdown` splits the trace into training steps (one optimizer
  launch per step) and reports per-kernel milliseconds per step, the number of
  launches, and the step's wall time vs. kernel-busy time (gaps = host/launch
  overhead);
* ``*_counter_collection.csv`` (``--pmc ...``): per-dispatch hardware counters.
  :func:`counter_summary` aggregates them per kernel and derives, where the
  counters are present, MFMA busy fraction (SQ_VALU_MFMA_BUSY_CYCLES over
  4 SIMDs × GRBM_GUI_ACTIVE), the wave-parked fraction (SQ_WAIT_ANY /
  SQ_WAVE_CYCLES: s_waitcnt / barrier stalls), issue-stall fraction
  (SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES) and LDS bank-conflict rate.

CLI::

    python -m replicann_amd.utils.profiling trace gpurun_out/prof/run_kernel_trace.csv --steps 3
    python -m replicann_amd.utils.profiling pmc gpurun_out/pmc/s1a_counter_collection.csv

(Counter collection with ``--pmc`` must run with ``--kernel-trace`` only — never
together with sys/runtime/hip traces on this pool.)
"""

from __future__ import annotations

import argparse
import csv
import re
import subprocess
from collections import defaultdict

CUS = 256
SIMDS_PER_CU = 4


def demangle(names):
    names = list(names)
    try:
        out = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True, check=True)
        return dict(zip(names, out.stdout.split("\n")))
    except Exception:  # c++filt missing: keep the mangled names
        return {n: n for n in names}


def short_name(name: str, width: int = 100) -> str:
    n = name.replace("(anonymous namespace)::", "").replace("rn_gemm_detail::", "")
    n = re.sub(r"^void ", "", n)
    n = re.sub(r"\(.*$", "", n)
    return n[:width]


def load_trace(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            wg = max(1, int(r.get("Workgroup_Size_X", 1) or 1))
            rows.append({"start": int(r["Start_Timestamp"]), "end": int(r["End_Timestamp"]),
                         "name": r["Kernel_Name"], "grid": int(r.get("Grid_Size_X", 0) or 0) // wg})
    dm = demangle({r["name"] for r in rows})
    for r in rows:
        r["name"] = dm.get(r["name"], r["name"])
    rows.sort(key=lambda r: r["start"])
    return rows


def step_breakdown(path, steps=3, marker=r"adamw|sgd_k|sgd_step"):
    """Average per-step kernel time over the last ``steps`` complete optimizer steps."""
    rows = load_trace(path)
    mk = re.compile(marker)
    ends = [i for i, r in enumerate(rows) if mk.search(r["name"])]
    if len(ends) < steps + 1:
        raise ValueError(f"only {len(ends)} optimizer launches in {path}")
    sel = rows[ends[-steps - 1] + 1: ends[-1] + 1]
    wall = (sel[-1]["end"] - sel[0]["start"]) / 1e6 / steps
    agg = defaultdict(lambda: [0, 0.0])
    for r in sel:
        k = short_name(r["name"])
        agg[k][0] += 1
        agg[k][1] += (r["end"] - r["start"]) / 1e6
    busy = sum(v[1] for v in agg.values()) / steps
    table = sorted(((t / steps, c / steps, k) for k, (c, t) in agg.items()), reverse=True)
    return {"wall_ms": wall, "busy_ms": busy, "launches": len(sel) / steps, "kernels": table}


def counter_summary(path):
    """Per-kernel sums of every counter column + derived utilisation metrics."""
    per = defaultdict(lambda: defaultdict(float))
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r.get("Kernel_Name", "?")
            cname = r.get("Counter_Name")
            if cname is None:
                continue
            per[name][cname] += float(r.get("Counter_Value", 0) or 0)
            per[name]["_n"] += 1
    dm = demangle(per.keys())
    out = []
    for name, c in per.items():
        d = {"kernel": short_name(dm.get(name, name)), **{k: v for k, v in c.items() if k != "_n"}}
        cyc = c.get("SQ_WAVE_CYCLES")
        if cyc:
            if "SQ_WAIT_ANY" in c:
                d["wait_any_frac"] = round(c["SQ_WAIT_ANY"] / cyc, 3)
            if "SQ_WAIT_INST_ANY" in c:
                d["issue_stall_frac"] = round(c["SQ_WAIT_INST_ANY"] / cyc, 3)
            if "SQ_ACTIVE_INST_ANY" in c:
                d["active_frac"] = round(c["SQ_ACTIVE_INST_ANY"] / cyc, 3)
        gui = c.get("GRBM_GUI_ACTIVE")
        if gui and "SQ_VALU_MFMA_BUSY_CYCLES" in c:
            # GRBM_GUI_ACTIVE is summed over the 8 XCDs; the busy counter over every SIMD
            d["mfma_busy"] = round(c["SQ_VALU_MFMA_BUSY_CYCLES"] / (gui / 8 * CUS * SIMDS_PER_CU), 3)
        if "SQ_LDS_BANK_CONFLICT" in c and c.get("SQ_LDS_IDX_ACTIVE"):
            d["lds_conflict_frac"] = round(c["SQ_LDS_BANK_CONFLICT"] / c["SQ_LDS_IDX_ACTIVE"], 3)
        out.append(d)
    return out


def main(argv=None):
    ap = argparse.ArgumentParser(prog="python -m replicann_amd.utils.profiling")
    sub = ap.add_subparsers(dest="cmd", required=True)
    t = sub.add_parser("trace")
    t.add_argument("csv")
    t.add_argument("--steps", type=int, default=3)
    t.add_argument("--top", type=int, default=40)
    p = sub.add_parser("pmc")
    p.add_argument("csv")
    a = ap.parse_args(argv)
    if a.cmd == "trace":
        r = step_breakdown(a.csv, a.steps)
        print(f"steps={a.steps}  wall/step={r['wall_ms']:.3f} ms  kernel-busy/step={r['busy_ms']:.3f} ms  "
              f"launches/step={r['launches']:.0f}")
        print(f"{'ms/step':>8} {'%':>5} {'n/step':>6}  kernel")
        for ms, n, k in r["kernels"][: a.top]:
            print(f"{ms:8.3f} {100 * ms / r['busy_ms']:5.1f} {n:6.0f}  {k}")
    else:
        import json
        for d in counter_summary(a.csv):
            print(json.dumps(d))


if __name__ == "__main__":
    main()
