import importlib
import os
import sys
from pathlib import Path

import pytest
import torch

ROOT = Path(__file__).resolve().parent.parent
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))

REF_SRC = Path("/root/reference/src")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) and the built _C.so")
    config.addinivalue_line("markers", "slow: long-running test")


def pytest_collection_modifyitems(config, items):
    have_gpu = torch.cuda.is_available()
    skip = pytest.mark.skip(reason="no GPU in this container")
    for it in items:
        if "gpu" in it.keywords and not have_gpu:
            it.add_marker(skip)


@pytest.fixture(scope="session")
def ref():
    """The reference package, imported read-only from /root/reference/src
    (test-only; never vendored).  Skips when absent."""
    if not REF_SRC.exists():
        pytest.skip("reference not mounted")
    saved = {k: v for k, v in sys.modules.items() if k == "replicann" or k.startswith("replicann.")}
    for k in saved:
        del sys.modules[k]
    sys.path.insert(0, str(REF_SRC))
    try:
        att = importlib.import_module("replicann.nn.attention")
        tr = importlib.import_module("replicann.arch.transformer")
    finally:
        sys.path.remove(str(REF_SRC))
        for k in [k for k in sys.modules if k == "replicann" or k.startswith("replicann.")]:
            del sys.modules[k]
        sys.modules.update(saved)

    class R:
        attention = att
        transformer = tr

    return R


@pytest.fixture
def cuda():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from replicann_amd import _ext
    assert _ext.available(), f"native extension failed to load: {_ext.load_error()}"
    return torch.device("cuda")
