"""N1 shipping hygiene (CPU): the loader refuses a ``_C.so`` built from other sources than this
tree's, the timing-only GEMM ablation kernels stay out of a default build, and the committed GEMM
tuning tables round-trip into the native autotuner cache."""

import json
from pathlib import Path

import pytest
import torch

from replicann_amd import _build, _ext

SO = Path(_build.OUT)


def test_source_digest_is_location_independent_and_content_sensitive(tmp_path):
    d = _build.source_digest()
    assert len(d) == 40 and d == _build.source_digest()
    assert "gemm_pk_dbg" not in {s.stem for s in _build._sources()} or _build.DEV


def test_stale_library_is_refused(tmp_path):
    fake = tmp_path / "_C.so"
    fake.write_bytes(b"\0")
    with pytest.raises(RuntimeError, match="no source stamp"):
        _ext.check_fresh(fake)
    fake.with_suffix(".srcstamp").write_text("0" * 40)
    with pytest.raises(RuntimeError, match="stale"):
        _ext.check_fresh(fake)
    fake.with_suffix(".srcstamp").write_text(_build.source_digest())
    _ext.check_fresh(fake)  # matching stamp: accepted


@pytest.mark.skipif(not SO.exists(), reason="extension not built")
def test_built_library_matches_tree():
    _ext.check_fresh(SO)


@pytest.mark.skipif(not SO.exists(), reason="extension not built")
def test_committed_tuning_tables_round_trip():
    from replicann_amd import tuning

    paths = sorted(tuning.DIR.glob("gemm_*.json"))
    if not paths:
        pytest.skip("no committed tuning tables")
    torch.ops.load_library(str(SO))
    for p in paths:
        entries = json.loads(p.read_text())
        assert entries and all({"M", "N", "K", "cfg", "split"} <= set(e) for e in entries)
        model = p.stem[len("gemm_"):]
        assert tuning.load_committed(model) == len(entries)
        table = json.loads(torch.ops.replicann.gemm_tuning_table())
        for e in entries:
            assert e in table
