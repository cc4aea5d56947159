"""Committed GEMM tuning tables (``gemm_<model>.json``): the per-shape kernel configs the runtime
autotuner measured for each BASELINE model's training step on an MI355X, loaded before the first
step so every process and every box runs the same kernels for those shapes (the autotuner still
times any shape a table does not cover).  Regenerate after a GEMM kernel change with
``scripts/gen_tuning_tables.sh`` on a GPU box (``bench.py`` writes the measured table of its run
to ``gpurun_out/gemm_tuning_<model>.json``).  ``REPLICANN_GEMM_TABLES=0`` skips loading."""

from __future__ import annotations

import json
import os
from pathlib import Path

DIR = Path(__file__).resolve().parent


def table_path(model: str) -> Path:
    return DIR / f"gemm_{model}.json"


def load_committed(model: str) -> int:
    """Load the committed table for ``model`` into the native autotuner cache (entries override
    nothing measured later: the cache is consulted first, so covered shapes are never re-timed).
    Returns the number of entries loaded (0 when there is no table or loading is disabled)."""
    if os.environ.get("REPLICANN_GEMM_TABLES", "1") == "0":
        return 0
    p = table_path(model)
    if not p.exists():
        return 0
    import torch

    from .. import _ext

    rows = json.loads(p.read_text())  # malformed file: fail loudly here, not as a silent partial parse
    _ext.ops()
    n = int(torch.ops.replicann.gemm_tuning_load(canonical(rows)))
    if n != len(rows):
        raise RuntimeError(f"{p}: the native loader took {n} of {len(rows)} entries")
    return n


KEYS = ("M", "N", "K", "ta", "tb", "act", "f32", "as", "epi", "cfg", "split")


def canonical(rows) -> str:
    """The exact compact form gemm_tuning_table() emits and gemm_tuning_load() parses (key order
    M, N, K, ta, tb, act, f32, as, epi, cfg, split; no spaces)."""
    return json.dumps([{k: int(r[k]) for k in KEYS} for r in rows], separators=(",", ":"))
