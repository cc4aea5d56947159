"""Full-size loss-trajectory check on the GPU: native bf16 path vs the plain-ATen fp32
reference math, same init and data.  Prints one JSON line per model.

    python scripts/check_trajectory.py --model gpt2-small vit-b16 --steps 8
    python scripts/check_trajectory.py --model gpt2-small --steps 100 --lr 1e-4 --threshold 0.02

``--threshold``: the largest allowed relative deviation |native - ref| / ref over the whole run
(exit status 1 beyond it), so the record carries its own pass/fail verdict.
"""

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from replicann_amd import _ext  # noqa: E402
from replicann_amd.training import TrainConfig, Trainer  # noqa: E402

DEFAULT_BATCH = {"vit-b16": 64, "resnet18": 128}


def run(model, steps, ref, batch, lr, warmup, sr=True):
    kw = dict(model=model, steps=steps, warmup_steps=warmup, lr=lr, log_every=10**9, batch_size=batch,
              dtype="fp32" if ref else "bf16", graph="off" if ref else "auto", stochastic_round=sr)
    if model.startswith("resnet"):
        kw.update(optimizer="sgd", lr=0.1)
    cfg = TrainConfig(**kw)
    losses = []
    if ref:
        with _ext.reference_path():
            t = Trainer(cfg)
            for _ in range(steps):
                losses.append(round(float(t.step()), 4))
    else:
        t = Trainer(cfg)
        for _ in range(steps):
            losses.append(round(float(t.step()), 4))
    del t
    return losses


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", nargs="+", default=["gpt2-small"])
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--lr", type=float, default=6e-4)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--threshold", type=float, default=None, help="max allowed relative deviation")
    ap.add_argument("--batch", type=int, default=None)
    ap.add_argument("--no-sr", action="store_true", help="nearest (not stochastic) rounding of the bf16 weights")
    a = ap.parse_args()
    ok = True
    for m in a.model:
        b = a.batch or DEFAULT_BATCH.get(m, 16)
        nat = run(m, a.steps, False, b, a.lr, a.warmup, sr=not a.no_sr)
        ref = run(m, a.steps, True, b, a.lr, a.warmup)
        dev = max(abs(x - y) for x, y in zip(nat, ref))
        rel = max(abs(x - y) / abs(y) for x, y in zip(nat, ref))
        passed = a.threshold is None or rel < a.threshold
        ok &= passed
        print(json.dumps({"model": m, "batch": b, "steps": a.steps, "stochastic_round": not a.no_sr, "lr": a.lr, "warmup": a.warmup,
                          "native_bf16": nat, "reference_fp32": ref, "max_abs_dev": round(dev, 4),
                          "max_rel_dev": round(rel, 5), "threshold": a.threshold, "pass": passed}), flush=True)
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
