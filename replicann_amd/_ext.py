"""Loader for the gfx950 extension (``_C.so``) and the device-path policy.

Two execution paths only: HIP kernels for tensors on the
GPU, plain ATen for CPU tensors.  On a GPU the native library is REQUIRED:
if ``_C.so`` is missing or fails to load, every op raises instead of silently
falling back to PyTorch.  (``REPLICANN_ALLOW_ATEN_FALLBACK=1`` exists only for
the stock-PyTorch comparison bench and is never set by tests.)
"""

from __future__ import annotations

import contextlib
import os
from pathlib import Path

import torch

# REPLICANN_SO: load another build of the library (A/B timing of two kernel revisions only; no
# staleness check for an explicitly named library)
_SO = Path(os.environ.get("REPLICANN_SO") or Path(__file__).resolve().parent / "_C.so")
_EXPLICIT = bool(os.environ.get("REPLICANN_SO"))


def check_fresh(so: Path = _SO) -> None:
    """Raise unless ``so`` was built from the sources in this tree (``_build.source_digest``).

    Only the source digest (the stamp's first line) is compared: the build's ``-D`` flags are
    recorded on its second line and describe the library, whatever the loading process's
    environment says.  Without a ``csrc/`` tree (an installed package ships ``_C.so`` and its stamp
    but no sources) there is nothing to compare against and the library is trusted."""
    from . import _build

    stamp = so.with_suffix(".srcstamp")
    if not stamp.exists():
        raise RuntimeError(f"{so} has no source stamp ({stamp.name}); rebuild with `python -m replicann_amd._build`")
    if not (_build.CSRC / "kernels").is_dir():
        return
    have = stamp.read_text().splitlines()[0].strip() if stamp.read_text().strip() else ""
    want = _build.source_digest()
    if have != want:
        raise RuntimeError(f"{so} is stale: it was built from other csrc/ sources than this tree's "
                           f"(stamp {have[:12]} != {want[:12]}); rebuild with "
                           "`python -m replicann_amd._build`")


def build_defs(so: Path = _SO) -> str:
    """The ``-D`` flags the loaded library was built with (from its stamp)."""
    stamp = so.with_suffix(".srcstamp")
    for line in (stamp.read_text().splitlines() if stamp.exists() else []):
        if line.startswith("defs:"):
            return line[5:].strip()
    return ""


_state = {"loaded": False, "error": None}
_ref = {"on": False}  # process-wide: autograd runs backward on its own device threads


def load() -> bool:
    if _state["loaded"]:
        return True
    if _state["error"] is not None:
        return False
    try:
        if not _SO.exists():
            raise FileNotFoundError(f"{_SO} not built (run `python -m replicann_amd._build`)")
        if not _EXPLICIT:
            check_fresh(_SO)
        torch.ops.load_library(str(_SO))
        _state["loaded"] = True
    except Exception as e:  # pragma: no cover - depends on build state
        _state["error"] = e
    return _state["loaded"]


def available() -> bool:
    return load()


def load_error():
    load()
    return _state["error"]


def ops():
    if not load():
        raise RuntimeError(f"replicann native extension unavailable: {_state['error']}")
    return torch.ops.replicann


def aten_fallback_allowed() -> bool:
    return os.environ.get("REPLICANN_ALLOW_ATEN_FALLBACK", "0") == "1"


@contextlib.contextmanager
def reference_path():
    """Run GPU tensors through the plain-ATen reference math instead of the HIP
    kernels (validation only: full-size fp32 loss-trajectory checks on the GPU)."""
    prev = _ref["on"]
    _ref["on"] = True
    try:
        yield
    finally:
        _ref["on"] = prev


def use_native(*tensors) -> bool:
    """True if this call must run on the HIP kernels.

    CPU tensors -> False (ATen path).  GPU tensors -> True, and the library
    must load; otherwise raise (no silent fallback on a GPU box).
    """
    dev = None
    for t in tensors:
        if isinstance(t, torch.Tensor):
            dev = t.device
            break
    if dev is None or dev.type != "cuda":
        return False
    if aten_fallback_allowed() or _ref["on"]:
        return False
    if not load():
        raise RuntimeError(
            f"GPU tensor passed to a replicann op but the gfx950 extension did not load: {_state['error']}"
        )
    return True
