"""Debug: LN e5m2 dY bitwise test — per step, per parameter, with and without the fp8 LM head."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import replicann_amd.ops.norm as norm_mod  # noqa: E402
from replicann_amd.models.gpt2 import GPT2, GPT2Config  # noqa: E402

os.environ["REPLICANN_DETERMINISTIC"] = "1"
cuda = torch.device("cuda")


def run(ln_q8, head, steps=3):
    torch.manual_seed(0)
    m = GPT2(GPT2Config.tiny(fp8=True, n_embd=256, vocab_size=2000, vocab_pad=2048, fp8_head=head)).to(cuda)
    for p in m.parameters():
        p.data = p.data.to(torch.bfloat16)
    idx = torch.randint(0, 2000, (4, 128), device=cuda, generator=torch.Generator(device=cuda).manual_seed(1))
    norm_mod.FP8_LN_Q8 = ln_q8
    out = []
    for _ in range(steps):
        m.zero_grad(set_to_none=True)
        loss = m(idx, idx)
        loss.backward()
        out.append((float(loss), {n: p.grad.clone() for n, p in m.named_parameters()}))
    return out


for head in (1, 0):
    a, b = run(True, head), run(False, head)
    for s, ((la, ga), (lb, gb)) in enumerate(zip(a, b)):
        diff = [n for n in ga if not torch.equal(ga[n], gb[n])]
        print(f"head={head} step {s + 1}: loss {la} vs {lb}; differing grads: {diff[:10]}")
