#!/usr/bin/env python
"""Headline benchmark (BASELINE.json): GPT-2-small bf16 DDP train-step samples/sec,
whole node, synthetic 1024-token sequences, random-init weights.

    python bench.py --gpus N --steps K --warmup W
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

One rank per GPU over RCCL.  W untimed warm-up steps, then EXACTLY K timed
steps bracketed by barrier + device synchronize on both sides; the elapsed
time is the MAX over ranks.  Every timed step is a full training step:
forward, loss, backward, bucketed gradient all-reduce, grad-norm clip and
fused AdamW update.  Rank 0 prints ONE JSON line.  Weak scaling: the per-GPU
micro-batch is fixed (default 64 x 1024 tokens: at N = 8 that is GPT-2's own
512-sequence global batch), the global batch is micro-batch × N.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

METRIC = "train-step samples/sec (whole node), GPT-2-small DDP at 1/2/4/8 MI355X"
OTHER_METRICS = {  # secondary BASELINE.json configs (same harness)
    "gpt2-medium": "train-step samples/sec (whole node), GPT-2-medium bf16",
    "gpt2-medium-fp8": "train-step samples/sec (whole node), GPT-2-medium fp8 forward GEMMs",
    "vit-b16": "train-step images/sec (whole node), ViT-B/16 bf16 DDP",
    "resnet18": "train-step images/sec (whole node), ResNet-18 bf16",
}
BASELINE_VALUE = None  # the reference publishes no number


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--model", default="gpt2-small")
    ap.add_argument("--batch", type=int, default=None,
                    help="per-GPU micro-batch (default: 64 sequences for GPT-2, i.e. GPT-2's own 512-sequence "
                         "global batch on 8 GPUs, sized for 288 GB HBM; 512 images ViT, 256 ResNet)")
    ap.add_argument("--seq", type=int, default=1024)
    ap.add_argument("--bucket-mb", type=float, default=64.0)
    ap.add_argument("--ddp", default="auto", choices=["auto", "on"],
                    help="on: run the data-parallel step (buckets, fp32 widening, collectives) even on 1 GPU")
    ap.add_argument("--comm", default="auto", choices=["auto", "native", "torch"],
                    help="collective back-end: native RCCL communicator (csrc/comm) or torch.distributed")
    ap.add_argument("--profile-steps", type=int, default=0, help="extra torch.profiler steps (not timed)")
    ap.add_argument("--graph", default="auto", choices=["auto", "on", "off"],
                    help="capture the whole training step as one hipGraph (auto: on for 1 process)")
    args = ap.parse_args()

    from replicann_amd import _ext
    from replicann_amd.training import TrainConfig, Trainer

    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    if world_env != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world_env}; using WORLD_SIZE", file=sys.stderr)
    if torch.cuda.is_available() and not _ext.available():
        raise RuntimeError(f"native extension missing: {_ext.load_error()}")

    is_lm = args.model.startswith("gpt2")
    if args.batch is None:  # ViT: 512 x 8 GPUs = ViT-B's 4096 global batch
        args.batch = 64 if is_lm else (512 if args.model.startswith("vit") else 256)
    cfg = TrainConfig(model=args.model, batch_size=args.batch, seq_len=args.seq, steps=10**9,
                      optimizer="adamw" if not args.model.startswith("resnet") else "sgd",
                      weight_decay=0.1 if not args.model.startswith("resnet") else 5e-5,
                      warmup_steps=10, lr=3e-4 if args.model.startswith("gpt2-medium") else 6e-4, bucket_mb=args.bucket_mb, log_every=10**9,
                      graph=args.graph, ddp=args.ddp, comm=args.comm)
    tr = Trainer(cfg)
    world = tr.world
    dev = tr.device

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)

    for i in range(args.warmup):
        loss = tr.step()
    sync()
    first_loss = float(loss) if args.warmup else float("nan")

    if world > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for i in range(args.steps):
        loss = tr.step()
    sync()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t)
    last_loss = float(loss)

    if args.profile_steps and tr.rank == 0:
        from torch.profiler import ProfilerActivity, profile
        with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
            for i in range(args.profile_steps):
                tr.step()
            sync()
        os.makedirs("gpurun_out", exist_ok=True)
        with open("gpurun_out/torch_profile.txt", "w") as f:
            f.write(prof.key_averages().table(sort_by="cuda_time_total", row_limit=60))

    ms = elapsed * 1000 / args.steps
    samples = cfg.batch_size * world * args.steps
    value = samples / elapsed
    out = {
        "metric": METRIC if args.model == "gpt2-small" else OTHER_METRICS.get(args.model, args.model),
        "value": round(value, 3),
        "unit": "samples/s" if is_lm else "images/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": (round(value / BASELINE_VALUE, 4) if BASELINE_VALUE else None),
        "dtype": "bf16",
        "data": ("synthetic (random bigram-chain token source, random-init weights)" if is_lm
                 else "synthetic (random images and labels, random-init weights)"),
        "config": {
            "model": args.model,
            "global_batch": cfg.batch_size * world,
            "micro_batch_per_gpu": cfg.batch_size,
            "seq_len": args.seq if is_lm else None,
            "parallelism": f"dp{world}",
            "tokens_per_s": round(value * args.seq, 1) if is_lm else None,
            "optimizer": ("fused AdamW" if cfg.optimizer == "adamw" else "fused SGD-momentum")
            + " (fp32 master) + grad-norm clip",
            "hipgraph": tr._graph is not None,
            "comm": (tr.ddp.comm.name if tr.ddp is not None else None),
            "loss_first_last": [round(first_loss, 4), round(last_loss, 4)],
        },
    }
    if tr.rank == 0:
        if dev.type == "cuda":  # the measured per-shape GEMM configs (runtime autotuner)
            os.makedirs("gpurun_out", exist_ok=True)
            with open(f"gpurun_out/gemm_tuning_{args.model}.json", "w") as f:
                f.write(torch.ops.replicann.gemm_tuning_table())
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
