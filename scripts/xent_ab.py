"""Fused LM cross-entropy row kernel A/B at the GPT-2-small b64 shape (65536 rows x 50304 padded
vocab, 50257 valid, bf16 logits overwritten by the gradient): v2 (default) vs the round-1 kernel
(REPLICANN_XENT=1).  Interleaved rounds in one process; reports ms and effective HBM TB/s
(one read + one write of the logits)."""

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from replicann_amd import _ext  # noqa: E402


def main():
    ops = _ext.ops()
    M, V, nv = 65536, 50304, 50257
    torch.manual_seed(0)
    base = (torch.randn(M, V, device="cuda") * 3).to(torch.bfloat16)
    work = torch.empty_like(base)
    tgt = torch.randint(0, nv, (M,), device="cuda")
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    res = {"2": [], "1": []}
    for _ in range(4):
        for k in ("2", "1"):
            os.environ["REPLICANN_XENT"] = k
            ts = []
            for _ in range(5):
                work.copy_(base)
                ev[0].record()
                ops.xent_fwd(work, tgt, nv, -100, True)
                ev[1].record()
                torch.cuda.synchronize()
                ts.append(ev[0].elapsed_time(ev[1]))
            res[k].append(min(ts))
    gb = 2 * M * V * 2 / 1e9
    out = {f"v{k}_ms": round(min(v), 4) for k, v in res.items()}
    out.update({f"v{k}_TBps": round(gb / min(v), 2) for k, v in res.items()})
    print(json.dumps(dict(M=M, V=V, **out)))


if __name__ == "__main__":
    main()
