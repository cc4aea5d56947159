"""GEMM autotuner table round trip (gemm_tuning_table -> gemm_tuning_load), the mechanism that makes
every data-parallel rank adopt rank 0's measured kernel choices (Trainer._tune).  CPU-only: the
table ops have no tensor arguments; needs the built extension."""

import json
from pathlib import Path

import pytest
import torch

SO = Path(__file__).resolve().parent.parent / "replicann_amd" / "_C.so"


@pytest.mark.skipif(not SO.exists(), reason="extension not built")
def test_tuning_table_round_trip():
    torch.ops.load_library(str(SO))
    entries = [dict(M=768, N=768, K=65536, ta=1, tb=0, act=0, f32=0, **{"as": 1}, epi=8, cfg=0, split=14),
               dict(M=65536, N=3072, K=768, ta=0, tb=1, act=5, f32=0, **{"as": 0}, epi=1, cfg=9, split=1)]
    assert torch.ops.replicann.gemm_tuning_load(json.dumps(entries, separators=(",", ":"))) == 2
    table = json.loads(torch.ops.replicann.gemm_tuning_table())
    for e in entries:
        assert e in table
    # loading a rank-0 table overrides a local pick for the same key
    e2 = dict(entries[1], cfg=1)
    assert torch.ops.replicann.gemm_tuning_load(json.dumps([e2], separators=(",", ":"))) == 1
    assert e2 in json.loads(torch.ops.replicann.gemm_tuning_table())


@pytest.mark.skipif(not SO.exists(), reason="extension not built")
def test_committed_tables_load_completely():
    """Every committed per-model table (replicann_amd/tuning/gemm_<model>.json) is loaded entry for
    entry by the native loader (load_committed raises on a partial parse)."""
    from replicann_amd import tuning

    torch.ops.load_library(str(SO))
    models = [p.stem[len("gemm_"):] for p in tuning.DIR.glob("gemm_*.json")]
    assert {"gpt2-small", "gpt2-medium", "gpt2-medium-fp8", "vit-b16", "resnet18"} <= set(models)
    for m in models:
        rows = json.loads(tuning.table_path(m).read_text())
        assert rows and tuning.load_committed(m) == len(rows)
        table = json.loads(torch.ops.replicann.gemm_tuning_table())
        for r in rows:
            assert {k: r[k] for k in tuning.KEYS} in table
