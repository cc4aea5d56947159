"""N21 entrypoints: ``python -m replicann train|eval`` / ``python -m replicann`` and the
``replicann.train`` / ``replicann.evaluate`` functions (CPU), plus packaging metadata."""

import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args):
    env = dict(os.environ, PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, "-m", *args], cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


def test_train_cli_and_checkpoint_eval(tmp_path):
    ck = str(tmp_path / "mlp.pt")
    out = _run("replicann", "train", "--model", "mlp", "--steps", "4", "--device", "cpu", "--batch-size", "16",
               "--checkpoint", ck)
    assert out["steps"] == 4 and out["final_loss"] is not None
    ev = _run("replicann", "eval", "--model", "mlp", "--device", "cpu", "--batch-size", "16", "--steps", "2",
              "--checkpoint", ck)
    assert ev["model"] == "mlp" and ev["loss"] > 0 and 0.0 <= ev["accuracy"] <= 1.0


def test_package_main_and_functions():
    out = _run("replicann", "--model", "mlp", "--steps", "2", "--device", "cpu", "--batch-size", "8")
    assert out["steps"] == 2
    import replicann
    res = replicann.train(model="mlp", steps=2, device="cpu", batch_size=8, log_every=100)
    assert res["steps"] == 2


def test_train_function_not_shadowed_by_a_module():
    """Round-1 bug: ``import replicann.train`` replaced the function with a CLI module."""
    import importlib
    import importlib.util

    import replicann
    assert importlib.util.find_spec("replicann.train") is None
    assert importlib.util.find_spec("replicann.eval") is None
    try:
        importlib.import_module("replicann.train")
    except ModuleNotFoundError:
        pass
    assert callable(replicann.train) and callable(replicann.evaluate)
    assert type(replicann.train).__name__ == "function"


def test_pyproject_declares_package_and_deps():
    import tomli
    with open(os.path.join(ROOT, "pyproject.toml"), "rb") as f:
        pp = tomli.load(f)
    proj = pp["project"]
    assert proj["name"] == "replicann" and proj["requires-python"].startswith(">=3.10")
    assert any(d.startswith("torch") for d in proj["dependencies"])
    assert proj["scripts"]["replicann"] == "replicann_amd.cli:main"
