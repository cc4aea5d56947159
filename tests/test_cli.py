"""N21 entrypoints: ``python -m replicann.train`` / ``python -m replicann.eval`` / ``python -m replicann``
and the ``replicann.train`` / ``replicann.evaluate`` functions (CPU)."""

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
    out = _run("replicann.train", "--model", "mlp", "--steps", "4", "--device", "cpu", "--batch-size", "16",
               "--checkpoint", ck)
    assert out["steps"] == 4 and out["final_loss"] is not None
    ev = _run("replicann.eval", "--model", "mlp", "--device", "cpu", "--batch-size", "16", "--steps", "2",
              "--checkpoint", ck)
    assert ev["model"] == "mlp" and ev["loss"] > 0 and 0.0 <= ev["accuracy"] <= 1.0


def test_package_main_and_functions():
    out = _run("replicann", "--model", "mlp", "--steps", "2", "--device", "cpu", "--batch-size", "8")
    assert out["steps"] == 2
    import replicann
    res = replicann.train(model="mlp", steps=2, device="cpu", batch_size=8, log_every=100)
    assert res["steps"] == 2
