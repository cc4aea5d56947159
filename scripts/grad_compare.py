"""First-step gradient comparison, native bf16 path vs the plain-ATen fp32 reference math (same
init, same batch): per parameter the relative L2 error, the norm ratio, the fraction of elements
whose sign differs (weighted by |g_ref|), and the fraction that are exactly zero in either.

    python scripts/grad_compare.py [--model gpt2-small] [--batch 16]
"""

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from replicann_amd import _ext  # noqa: E402
from replicann_amd.training import TrainConfig, Trainer  # noqa: E402


def grads(model, batch, ref, seq):
    cfg = TrainConfig(model=model, steps=1, batch_size=batch, seq_len=seq, log_every=10**9,
                      dtype="fp32" if ref else "bf16", graph="off")
    ctx = _ext.reference_path() if ref else torch.enable_grad()
    with ctx:
        t = Trainer(cfg)
        t.opt.zero_grad()
        x, y = next(t.data)
        loss = t.net(x, y)
        loss.backward()
        if t.ddp is not None:
            t.ddp.finish()
        out = {n: p.grad.detach().float().clone() for n, p in t.model.named_parameters()}
        norm = float(t.flat.grad.float().norm())
    return float(loss), out, norm


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="gpt2-small")
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--seq", type=int, default=1024)
    a = ap.parse_args()
    ln, gn, nn_ = grads(a.model, a.batch, False, a.seq)
    lr_, gr, nr = grads(a.model, a.batch, True, a.seq)
    print(json.dumps({"loss_native": ln, "loss_ref": lr_, "flat_grad_norm_native": nn_, "flat_grad_norm_ref": nr}))
    for n in gr:
        g, r = gn[n], gr[n]
        err = float((g - r).norm() / (r.norm() + 1e-30))
        ratio = float(g.norm() / (r.norm() + 1e-30))
        w = r.abs()
        flip = float((w * ((g.sign() != r.sign()) & (r != 0)).float()).sum() / (w.sum() + 1e-30))
        zn = float((g == 0).float().mean())
        zr = float((r == 0).float().mean())
        print(json.dumps({"param": n, "rel_err": round(err, 5), "norm_ratio": round(ratio, 5),
                          "signflip_w": round(flip, 5), "zero_native": round(zn, 5), "zero_ref": round(zr, 5),
                          "ref_norm": float(r.norm())}), flush=True)


if __name__ == "__main__":
    main()
