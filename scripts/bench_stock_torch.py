"""Comparison baseline (BASELINE.md row "stock PyTorch-ROCm"): the same GPT-2-small
training step written the stock way — nn.Linear (hipBLASLt), fp32 params under
bf16 autocast, F.scaled_dot_product_attention, torch's fused AdamW with grad
clipping, torch DDP for N>1.  Same timing protocol and JSON line as bench.py."""

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
    def __init__(self, E, H):
        super().__init__()
        self.ln_1, self.ln_2 = nn.LayerNorm(E), nn.LayerNorm(E)
        self.c_attn, self.c_proj = nn.Linear(E, 3 * E), nn.Linear(E, E)
        self.fc, self.fc2 = nn.Linear(E, 4 * E), nn.Linear(4 * E, E)
        self.H = H

    def forward(self, x):
        B, T, E = x.shape
        q, k, v = self.c_attn(self.ln_1(x)).view(B, T, 3, self.H, E // self.H).unbind(2)
        a = F.scaled_dot_product_attention(q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2), is_causal=True)
        x = x + self.c_proj(a.transpose(1, 2).reshape(B, T, E))
        return x + self.fc2(F.gelu(self.fc(self.ln_2(x)), approximate="tanh"))


class GPT(nn.Module):
    def __init__(self, L=12, E=768, H=12, V=50304, T=1024):
        super().__init__()
        self.wte, self.wpe = nn.Embedding(V, E), nn.Embedding(T, E)
        self.h = nn.ModuleList(Block(E, H) for _ in range(L))
        self.ln_f = nn.LayerNorm(E)

    def forward(self, idx, tgt):
        x = self.wte(idx) + self.wpe(torch.arange(idx.shape[1], device=idx.device))
        for b in self.h:
            x = b(x)
        logits = self.ln_f(x) @ self.wte.weight.t()
        return F.cross_entropy(logits.float().reshape(-1, logits.shape[-1])[:, :50257], tgt.reshape(-1))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=16)
    a = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", 1))
    rank = int(os.environ.get("RANK", 0))
    lr_ = int(os.environ.get("LOCAL_RANK", 0))
    torch.cuda.set_device(lr_)
    if world > 1:
        dist.init_process_group("nccl")
    torch.manual_seed(0)
    model = GPT().cuda()
    net = nn.parallel.DistributedDataParallel(model, device_ids=[lr_]) if world > 1 else model
    opt = torch.optim.AdamW(model.parameters(), lr=6e-4, betas=(0.9, 0.95), weight_decay=0.1, fused=True)
    data = torch.randint(0, 50257, (a.batch, 1025), device="cuda")

    def step():
        opt.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = net(data[:, :-1], data[:, 1:])
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
        print(json.dumps({"metric": "stock PyTorch-ROCm GPT-2-small train samples/s", "value": round(v, 2),
                          "ms_per_step": round(el * 1000 / a.steps, 2), "n_gpus": world, "batch": a.batch,
                          "loss": float(loss)}))


if __name__ == "__main__":
    main()
