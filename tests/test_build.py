"""N1 shipping hygiene (CPU): the loader refuses a ``_C.so`` built from other sources than this
tree's, the timing-only GEMM ablation kernels stay out of a default build, and the committed GEMM
tuning tables round-trip into the native autotuner cache."""

import json
import shutil
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


def test_stamp_flags_do_not_depend_on_the_loading_environment(tmp_path, monkeypatch):
    """A library built with debug checks still loads in a process without REPLICANN_CHECK: the
    stamp's first line is the source digest, the build defs are recorded, not re-derived."""
    fake = tmp_path / "_C.so"
    fake.write_bytes(b"\0")
    fake.with_suffix(".srcstamp").write_text(f"{_build.source_digest()}\ndefs: -DREPLICANN_CHECK=1\n")
    _ext.check_fresh(fake)
    assert _ext.build_defs(fake) == "-DREPLICANN_CHECK=1"
    assert _build.stamp_text().splitlines()[0] == _build.source_digest()


def test_installed_package_without_sources_is_trusted(tmp_path, monkeypatch):
    """A non-editable install ships _C.so + its stamp but no csrc/: nothing to compare, load it."""
    fake = tmp_path / "_C.so"
    fake.write_bytes(b"\0")
    fake.with_suffix(".srcstamp").write_text("0" * 40 + "\ndefs: \n")
    monkeypatch.setattr(_build, "CSRC", tmp_path / "no_csrc")
    _ext.check_fresh(fake)


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


@pytest.mark.skipif(not SO.exists() or shutil.which("nm") is None, reason="extension not built / no nm")
def test_release_library_has_no_ablation_kernels():
    """The timing-only GEMM ablations (DBG != 0: operand DMA out of range, every tile at (0,0) —
    WRONG outputs by design) exist only in a REPLICANN_DEV build; a release _C.so must not carry
    a single instantiation of them."""
    import re
    import subprocess

    stamp = SO.with_suffix(".srcstamp")
    if stamp.exists() and "-DREPLICANN_DEV=1" in stamp.read_text():
        pytest.skip("developer build")
    out = subprocess.run(["nm", "-DC", "--defined-only", str(SO)], capture_output=True, text=True, check=True).stdout
    pk = re.findall(r"gemm_pk<([^>]*)>", out)
    w1 = re.findall(r"gemm_w1<([^>]*)>", out)
    assert pk and w1, "expected the production GEMM kernels in the library"
    # template argument 5 of gemm_pk and 4 of gemm_w1 is DBG
    assert all(a.split(", ")[5] == "0" for a in pk), sorted({a for a in pk if a.split(", ")[5] != "0"})
    assert all(a.split(", ")[4] == "0" for a in w1), sorted({a for a in w1 if a.split(", ")[4] != "0"})
