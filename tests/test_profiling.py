"""CPU tests of the rocprofv3 CSV analysis (replicann_amd.utils.profiling)."""

import csv

from replicann_amd.utils import profiling

TRACE_COLS = ["Kind", "Kernel_Name", "Start_Timestamp", "End_Timestamp", "Workgroup_Size_X", "Grid_Size_X"]


def _write_trace(path, rows):
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(TRACE_COLS)
        for r in rows:
            w.writerow(r)


def test_step_breakdown(tmp_path):
    rows, t = [], 0
    for _step in range(4):  # gemm 100 us, ln 10 us, adamw 50 us per step, 5 us gaps
        for name, d in (("gemm_k", 100_000), ("ln_fwd_k", 10_000), ("adamw_k", 50_000)):
            rows.append(["KERNEL_DISPATCH", name, t, t + d, 256, 256 * 64])
            t += d + 5_000
    p = tmp_path / "run_kernel_trace.csv"
    _write_trace(p, rows)
    r = profiling.step_breakdown(str(p), steps=3)
    assert abs(r["busy_ms"] - 0.16) < 1e-9
    assert r["launches"] == 3
    assert r["kernels"][0][2] == "gemm_k" and abs(r["kernels"][0][0] - 0.1) < 1e-9
    assert r["wall_ms"] > r["busy_ms"]


def test_counter_summary(tmp_path):
    p = tmp_path / "c.csv"
    with open(p, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Kernel_Name", "Counter_Name", "Counter_Value"])
        for cname, v in (("SQ_WAVE_CYCLES", 1000), ("SQ_WAIT_ANY", 250), ("SQ_WAIT_INST_ANY", 100),
                         ("SQ_LDS_BANK_CONFLICT", 5), ("SQ_LDS_IDX_ACTIVE", 50)):
            w.writerow(["k1", cname, v])
    (d,) = profiling.counter_summary(str(p))
    assert d["wait_any_frac"] == 0.25 and d["issue_stall_frac"] == 0.1 and d["lds_conflict_frac"] == 0.1
