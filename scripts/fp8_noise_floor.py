"""fp8 numerics against a noise floor: GPT-2-medium, three runs of ``steps`` steps at
micro-batch ``batch`` x 1024, lr 1e-4 (warm-up 10), the same init (seed 7):

  bf16_a   the bf16 model on the synthetic token stream of seed 7
  bf16_b   the bf16 model on the stream of ANOTHER data seed (same source language, other sequences):
           the step-to-step deviation two equally valid bf16 runs show — the noise floor
  fp8      the fp8 model on the stream of seed 7; before every step the same batch is also scored
           under no_grad, where the fp8 model's LM head runs in bf16 (its GEMMs still e4m3, on scratch
           copies of the delayed scales: the training state is untouched, tests/test_fp8_inference_gpu.py)
           — that loss separates the fp8 head's logits quantisation from trajectory divergence.

Reported per window (steps 1-10, 11-50, 51-steps): mean and max relative deviation of fp8 from bf16_a,
of fp8-with-bf16-head from bf16_a, and of bf16_b from bf16_a; the verdict's criterion is fp8's windowed
deviation <= 1.5x the bf16 seed-to-seed deviation.  One JSON line per step, then per window, then a summary.

    python scripts/fp8_noise_floor.py [steps] [batch] [lr]"""

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from replicann_amd.training import TrainConfig, Trainer  # noqa: E402
from replicann_amd.utils.data import SyntheticLM  # noqa: E402


class Peek:
    """The trainer's data source with a look-ahead: the batch the next step will take."""

    def __init__(self, src):
        self.src, self.buf = src, None

    def peek(self):
        if self.buf is None:
            self.buf = next(self.src)
        return self.buf

    def __next__(self):
        b = self.peek()
        self.buf = None
        return b

    def __iter__(self):
        return self

    def state_dict(self):
        return self.src.state_dict()

    def load_state_dict(self, sd):
        self.src.load_state_dict(sd)


def run(model, steps, batch, lr, data_seed=None, head_probe=False):
    cfg = TrainConfig(model=model, batch_size=batch, seq_len=1024, steps=steps, lr=lr, warmup_steps=10,
                      weight_decay=0.1, log_every=10**9, seed=7)
    tr = Trainer(cfg)
    if data_seed is not None:
        tr.data = SyntheticLM(batch, 1024, tr.model.config.vocab_size, tr.device, seed=data_seed * 1000)
    tr.data = Peek(tr.data)
    out, probe = [], []
    for _ in range(steps):
        if head_probe:
            x, y = tr.data.peek()
            with torch.no_grad():
                probe.append(float(tr.model(x, y)))
        out.append(float(tr.step()))
        print(json.dumps({"run": model + ("" if data_seed is None else f"/data{data_seed}"), "step": len(out),
                          "loss": round(out[-1], 5), **({"bf16_head": round(probe[-1], 5)} if head_probe else {})}),
              flush=True)
    del tr
    torch.cuda.empty_cache()
    return out, probe


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    batch = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    lr = float(sys.argv[3]) if len(sys.argv) > 3 else 1e-4
    a, _ = run("gpt2-medium", steps, batch, lr)
    b, _ = run("gpt2-medium", steps, batch, lr, data_seed=8)
    f, fh = run("gpt2-medium-fp8", steps, batch, lr, head_probe=True)
    rel = lambda u, v: [abs(x - y) / abs(y) for x, y in zip(u, v)]  # noqa: E731
    d_f8, d_f8h, d_bb = rel(f, a), rel(fh, a), rel(b, a)
    summary = {"summary": True, "steps": steps, "batch": batch, "lr": lr, "windows": []}
    ok = True
    for lo, hi in ((1, 10), (11, 50), (51, steps)):
        if lo > steps:
            continue
        w = slice(lo - 1, min(hi, steps))
        row = {"window": f"{lo}-{min(hi, steps)}"}
        for name, d in (("fp8", d_f8), ("fp8_bf16head", d_f8h), ("bf16_seed", d_bb)):
            row[name + "_mean"] = round(sum(d[w]) / len(d[w]), 5)
            row[name + "_max"] = round(max(d[w]), 5)
        row["ratio_mean"] = round(row["fp8_mean"] / max(row["bf16_seed_mean"], 1e-9), 3)
        ok = ok and row["ratio_mean"] <= 1.5
        print(json.dumps(row), flush=True)
        summary["windows"].append(row)
    summary["fp8_within_1p5x_noise_floor"] = ok
    print(json.dumps(summary), flush=True)


if __name__ == "__main__":
    main()
