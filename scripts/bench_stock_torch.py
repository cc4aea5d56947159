"""Comparison baseline (BASELINE.md column "stock PyTorch-ROCm"): the same training
steps bench.py runs, written the stock way — nn.Linear / nn.Conv2d (hipBLASLt,
MIOpen), fp32 params under bf16 autocast, F.scaled_dot_product_attention,
nn.LayerNorm / nn.BatchNorm2d, torch's fused AdamW (SGD-momentum for ResNet-18)
with grad clipping, torch DDP for N>1.  Same timing protocol as bench.py.

    python scripts/bench_stock_torch.py --model {gpt2-small,gpt2-medium,vit-b16,resnet18} [--batch B]
"""

import argparse
import json
import math
import os
import time

import torch
import torch.distributed as dist
import torch.nn as nn
import torch.nn.functional as F


class Block(nn.Module):
    def __init__(self, E, H, causal=True):
        super().__init__()
        self.causal = causal
        self.ln_1, self.ln_2 = nn.LayerNorm(E), nn.LayerNorm(E)
        self.c_attn, self.c_proj = nn.Linear(E, 3 * E), nn.Linear(E, E)
        self.fc, self.fc2 = nn.Linear(E, 4 * E), nn.Linear(4 * E, E)
        self.H = H

    def forward(self, x):
        B, T, E = x.shape
        q, k, v = self.c_attn(self.ln_1(x)).view(B, T, 3, self.H, E // self.H).unbind(2)
        a = F.scaled_dot_product_attention(q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2), is_causal=self.causal)
        x = x + self.c_proj(a.transpose(1, 2).reshape(B, T, E))
        return x + self.fc2(F.gelu(self.fc(self.ln_2(x)), approximate="tanh"))


class GPT(nn.Module):
    def __init__(self, L=12, E=768, H=12, V=50304, T=1024, causal=True):
        super().__init__()
        self.wte, self.wpe = nn.Embedding(V, E), nn.Embedding(T, E)
        self.h = nn.ModuleList(Block(E, H) for _ in range(L))
        self.ln_f = nn.LayerNorm(E)
        nn.init.normal_(self.wte.weight, std=0.02)
        nn.init.normal_(self.wpe.weight, std=0.01)

    def forward(self, idx, tgt):
        x = self.wte(idx) + self.wpe(torch.arange(idx.shape[1], device=idx.device))
        for b in self.h:
            x = b(x)
        logits = self.ln_f(x) @ self.wte.weight.t()
        return F.cross_entropy(logits.float().reshape(-1, logits.shape[-1])[:, :50257], tgt.reshape(-1))


class ViT(nn.Module):
    """ViT-B/16: 16x16 patch-embed conv, CLS token, 12 pre-LN blocks, 1000-way head."""

    def __init__(self, L=12, E=768, H=12, classes=1000, img=224, patch=16):
        super().__init__()
        self.patch = nn.Conv2d(3, E, patch, patch)
        n = (img // patch) ** 2
        self.cls = nn.Parameter(torch.zeros(1, 1, E))
        self.pos = nn.Parameter(torch.randn(1, n + 1, E) * 0.02)
        self.h = nn.ModuleList(Block(E, H, causal=False) for _ in range(L))
        self.ln_f, self.head = nn.LayerNorm(E), nn.Linear(E, classes)

    def forward(self, x, y):
        x = self.patch(x).flatten(2).transpose(1, 2)
        x = torch.cat([self.cls.expand(x.shape[0], -1, -1), x], 1) + self.pos
        for b in self.h:
            x = b(x)
        return F.cross_entropy(self.head(self.ln_f(x[:, 0])).float(), y)


class Basic(nn.Module):
    def __init__(self, cin, cout, stride):
        super().__init__()
        self.c1, self.b1 = nn.Conv2d(cin, cout, 3, stride, 1, bias=False), nn.BatchNorm2d(cout)
        self.c2, self.b2 = nn.Conv2d(cout, cout, 3, 1, 1, bias=False), nn.BatchNorm2d(cout)
        self.sc = None
        if stride != 1 or cin != cout:
            self.sc = nn.Sequential(nn.Conv2d(cin, cout, 1, stride, bias=False), nn.BatchNorm2d(cout))

    def forward(self, x):
        y = self.b2(self.c2(F.relu(self.b1(self.c1(x)))))
        return F.relu(y + (x if self.sc is None else self.sc(x)))


class ResNet18(nn.Module):
    def __init__(self, classes=1000):
        super().__init__()
        self.stem = nn.Sequential(nn.Conv2d(3, 64, 7, 2, 3, bias=False), nn.BatchNorm2d(64), nn.ReLU(),
                                  nn.MaxPool2d(3, 2, 1))
        layers, cin = [], 64
        for cout, s in [(64, 1), (128, 2), (256, 2), (512, 2)]:
            layers += [Basic(cin, cout, s), Basic(cout, cout, 1)]
            cin = cout
        self.layers = nn.Sequential(*layers)
        self.fc = nn.Linear(512, classes)

    def forward(self, x, y):
        x = self.layers(self.stem(x))
        return F.cross_entropy(self.fc(x.mean((2, 3))).float(), y)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=None)
    ap.add_argument("--model", default="gpt2-small", choices=["gpt2-small", "gpt2-medium", "vit-b16", "resnet18"])
    a = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", 1))
    rank = int(os.environ.get("RANK", 0))
    lr_ = int(os.environ.get("LOCAL_RANK", 0))
    torch.cuda.set_device(lr_)
    if world > 1:
        dist.init_process_group("nccl")
    torch.manual_seed(0)
    lm = a.model.startswith("gpt2")
    if a.batch is None:
        a.batch = 64 if lm else 256
    if a.model == "gpt2-small":
        model = GPT().cuda()
    elif a.model == "gpt2-medium":
        model = GPT(L=24, E=1024, H=16).cuda()
    elif a.model == "vit-b16":
        model = ViT().cuda()
    else:
        model = ResNet18().cuda().to(memory_format=torch.channels_last)
    net = nn.parallel.DistributedDataParallel(model, device_ids=[lr_]) if world > 1 else model
    if a.model == "resnet18":
        opt = torch.optim.SGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=5e-5, foreach=True)
    else:
        opt = torch.optim.AdamW(model.parameters(), lr=6e-4, betas=(0.9, 0.95), weight_decay=0.1, fused=True)
    if lm:
        data = torch.randint(0, 50257, (a.batch, 1025), device="cuda")
        inp, tgt = data[:, :-1], data[:, 1:]
    else:
        inp = torch.randn(a.batch, 3, 224, 224, device="cuda")
        if a.model == "resnet18":
            inp = inp.to(memory_format=torch.channels_last)
        tgt = torch.randint(0, 1000, (a.batch,), device="cuda")

    def step():
        opt.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = net(inp, tgt)
        loss.backward()
        torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
        opt.step()
        return loss

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        loss = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    v = a.batch * world * a.steps / el
    if rank == 0:
        print(json.dumps({"metric": f"stock PyTorch-ROCm {a.model} train samples/s", "value": round(v, 2),
                          "ms_per_step": round(el * 1000 / a.steps, 2), "n_gpus": world, "batch": a.batch,
                          "loss": float(loss)}))


if __name__ == "__main__":
    main()
