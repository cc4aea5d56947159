"""GPT-2-medium fp8 vs bf16 loss trajectory (same seed, same synthetic token stream, same
schedule): 50 steps at micro-batch 16 x 1024, lr 1e-4 by default (warm-up 10; argv: steps batch lr).  Writes one JSON line per
step and a summary line with the max relative deviation of the fp8 loss from the bf16 loss."""

import json
import sys
import os

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from replicann_amd.training import TrainConfig, Trainer  # noqa: E402


def run(model, steps, batch, lr):
    cfg = TrainConfig(model=model, batch_size=batch, seq_len=1024, steps=steps, lr=lr, warmup_steps=10,
                      weight_decay=0.1, log_every=10**9, seed=7)
    tr = Trainer(cfg)
    out = [float(tr.step()) for _ in range(steps)]
    # held-out loss of the trained model in eval mode (the next 4 batches of the same stream for both runs): the
    # fp8 model's LM head runs in bf16 there, so this separates training quality from the fp8 head's logits
    # noise in the training loss (E[lse(z + e)] > lse(z))
    tr.model.eval()
    with torch.no_grad():
        ev = sum(float(tr.model(*(t.cuda() for t in next(tr.data)))) for _ in range(4)) / 4
    tr.model.train()
    del tr
    torch.cuda.empty_cache()
    return out, ev


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    batch = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    lr = float(sys.argv[3]) if len(sys.argv) > 3 else 1e-4
    bf, ev_bf = run("gpt2-medium", steps, batch, lr)
    f8, ev_f8 = run("gpt2-medium-fp8", steps, batch, lr)
    dev = [abs(a - b) / abs(b) for a, b in zip(f8, bf)]
    for i, (a, b, d) in enumerate(zip(bf, f8, dev)):
        print(json.dumps({"step": i + 1, "bf16": round(a, 5), "fp8": round(b, 5), "rel_dev": round(d, 5)}))
    print(json.dumps({"summary": True, "steps": steps, "batch": batch, "lr": lr, "max_rel_dev": round(max(dev), 5),
                      "final_bf16": round(bf[-1], 5), "final_fp8": round(f8[-1], 5),
                      "eval_bf16": round(ev_bf, 5), "eval_fp8": round(ev_f8, 5),
                      "eval_rel_dev": round(abs(ev_f8 - ev_bf) / abs(ev_bf), 5)}))


if __name__ == "__main__":
    main()
