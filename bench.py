#!/usr/bin/env python
"""Headline benchmark (BASELINE.json): GPT-2-small bf16 DDP train-step samples/sec,
whole node, synthetic 1024-token sequences, random-init weights.

    python bench.py --gpus N --steps K --warmup W
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

One rank per GPU over RCCL.  Without an external launcher (no WORLD_SIZE in the
environment) ``--gpus N`` with N > 1 makes this process a launcher: it never touches
the GPU, spawns N fresh worker processes of itself (RANK / LOCAL_RANK / WORLD_SIZE /
MASTER_ADDR=127.0.0.1 / a free MASTER_PORT), forwards rank 0's output and exits with
the worst worker exit code.  A worker whose process group or communicator does not
span exactly ``--gpus`` ranks exits non-zero instead of reporting a number.
W untimed warm-up steps, then EXACTLY K timed
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

METRIC = "train-step samples/sec (whole node), GPT-2-small DDP at 1/2/4/8 MI355X"
OTHER_METRICS = {  # secondary BASELINE.json configs (same harness)
    "gpt2-medium": "train-step samples/sec (whole node), GPT-2-medium bf16",
    "gpt2-medium-fp8": "train-step samples/sec (whole node), GPT-2-medium fp8 forward GEMMs",
    "vit-b16": "train-step images/sec (whole node), ViT-B/16 bf16 DDP",
    "resnet18": "train-step images/sec (whole node), ResNet-18 bf16",
    "mlp": "train-step samples/sec, 2-layer MLP on MNIST-shaped tensors (CPU plumbing config)",
}
BASELINE_VALUE = None  # the reference publishes no number


def parse_args(argv=None):
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
    ap.add_argument("--reduce-dtype", default="rsag", choices=["rsag", "fp32", "bf16"],
                    help="DDP gradient sum: rsag = fp32 reduce-scatter + bf16 all-gather of the reduced shards "
                         "(exact sum, one rounding, 0.75x the bytes of fp32); fp32 all-reduce; bf16 in place")
    ap.add_argument("--ddp-schedule", default="auto", choices=["auto", "eager", "window", "end"],
                    help="when a ready gradient bucket's collective is issued: at once, beside the next attention "
                         "backward (the persistent GEMMs own every CU), or after the backward")
    ap.add_argument("--ddp", default="auto", choices=["auto", "on"],
                    help="on: run the data-parallel step (buckets, fp32 widening, collectives) even on 1 GPU")
    ap.add_argument("--comm", default="auto", choices=["auto", "native", "torch", "proxy"],
                    help="collective back-end: native RCCL communicator (csrc/comm), torch.distributed, or "
                         "proxy (1-GPU stand-in with RCCL's CU/HBM footprint, for interference measurements)")
    ap.add_argument("--profile-steps", type=int, default=0, help="extra torch.profiler steps (not timed)")
    ap.add_argument("--graph", default="auto", choices=["auto", "on", "off"],
                    help="capture the whole training step as one hipGraph (auto: on for 1 process)")
    ap.add_argument("--device", default=None, help="cpu: run the same harness on the CPU/gloo path (tests)")
    ap.add_argument("--ce-chunk", type=int, default=0,
                    help="GPT-2: LM head + loss over token chunks of this size (0: whole batch)")
    return ap.parse_args(argv)


def launch_workers(args, argv):
    """``--gpus N`` without an external launcher: N fresh worker processes of this script, one
    per GPU (the parent imports nothing that initialises the GPU and never execs)."""
    import signal
    import socket
    import subprocess

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv], env=env,
                                      stdout=None if r == 0 else subprocess.DEVNULL))
    rcs = [None] * len(procs)
    while any(rc is None for rc in rcs):
        for i, p in enumerate(procs):
            if rcs[i] is None:
                rcs[i] = p.poll()
        if any(rc not in (None, 0) for rc in rcs):  # one rank failed: the others would hang in a collective
            for i, p in enumerate(procs):
                if rcs[i] is None:
                    p.send_signal(signal.SIGTERM)
            for i, p in enumerate(procs):
                if rcs[i] is None:
                    try:
                        rcs[i] = p.wait(timeout=30)
                    except subprocess.TimeoutExpired:
                        p.kill()
                        rcs[i] = p.wait()
            break
        time.sleep(0.2)
    bad = [rc for rc in rcs if rc]
    return (max(abs(rc) for rc in bad) or 1) if bad else 0


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse_args(argv)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_workers(args, argv))

    import torch
    import torch.distributed as dist

    from replicann_amd import _ext
    from replicann_amd.training import TrainConfig, Trainer

    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    if world_env != args.gpus:
        print(f"error: --gpus {args.gpus} but the launcher started WORLD_SIZE={world_env} ranks", file=sys.stderr)
        sys.exit(3)
    if torch.cuda.is_available() and args.device != "cpu" and not _ext.available():
        raise RuntimeError(f"native extension missing: {_ext.load_error()}")

    is_lm = args.model.startswith("gpt2")
    if args.batch is None:  # ViT: 512 x 8 GPUs = ViT-B's 4096 global batch
        args.batch = 64 if is_lm else (512 if args.model.startswith("vit") else 256)
    cfg = TrainConfig(model=args.model, batch_size=args.batch, seq_len=args.seq, steps=10**9,
                      optimizer="adamw" if not args.model.startswith("resnet") else "sgd",
                      weight_decay=0.1 if not args.model.startswith("resnet") else 5e-5,
                      warmup_steps=10, lr=3e-4 if args.model.startswith("gpt2-medium") else 6e-4, bucket_mb=args.bucket_mb,
                      reduce_dtype=args.reduce_dtype, ddp_schedule=args.ddp_schedule, log_every=10**9,
                      graph=args.graph, ddp=args.ddp, comm=args.comm, device=args.device,
                      model_kwargs={"ce_chunk": args.ce_chunk} if (is_lm and args.ce_chunk) else {})
    tr = Trainer(cfg)
    world = tr.world
    dev = tr.device
    comm_world = tr.ddp.comm.world if tr.ddp is not None else 1
    if world != args.gpus or (args.comm != "proxy" and comm_world != world):
        print(f"error: --gpus {args.gpus} but the process group has {world} ranks and the "
              f"communicator {comm_world}", file=sys.stderr)
        sys.exit(3)

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
    rank_ms = [round(elapsed * 1000 / max(args.steps, 1), 3)]
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t)
        rank_ms = [None] * world
        dist.all_gather_object(rank_ms, round((t1 - t0) * 1000 / max(args.steps, 1), 3))
    last_loss = float(loss)
    # after the timed loop: one untimed, phase-timed eager step of the data-parallel path, so a first
    # multi-GPU record says where its time went (exposed comm, collectives / bytes, schedule, spread)
    diag = ddp_diagnostics(tr, world, rank_ms, sync) if tr.ddp is not None else None

    if args.profile_steps and tr.rank == 0:
        from torch.profiler import ProfilerActivity, profile
        with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
            for i in range(args.profile_steps):
                tr.step()
            sync()
        os.makedirs("gpurun_out", exist_ok=True)
        with open("gpurun_out/torch_profile.txt", "w") as f:
            f.write(prof.key_averages().table(sort_by="cuda_time_total", row_limit=60))

    graphs = [tr._graph is not None]
    if world > 1:  # per-rank capture state (every rank must run the same step form)
        graphs = [None] * world
        dist.all_gather_object(graphs, tr._graph is not None)

    ms = elapsed * 1000 / args.steps
    samples = cfg.batch_size * world * args.steps
    value = samples / elapsed
    out = {
        "metric": METRIC if args.model == "gpt2-small" else OTHER_METRICS.get(args.model, args.model),
        "value": round(value, 3),
        "unit": "samples/s" if (is_lm or args.model == "mlp") else "images/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": (round(value / BASELINE_VALUE, 4) if BASELINE_VALUE else None),
        "dtype": precision(tr.model),
        "data": ("synthetic (random bigram-chain token source, random-init weights)" if is_lm
                 else "synthetic (random MNIST-shaped tensors and labels, random-init weights)" if args.model == "mlp"
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
            "hipgraph": graphs,
            "comm": (tr.ddp.comm.name if tr.ddp is not None else None),
            "comm_world": comm_world,
            "grad_reduce_dtype": args.reduce_dtype if tr.ddp is not None else None,
            "ddp_schedule": args.ddp_schedule if tr.ddp is not None else None,
            "gemm_cu_reserve": (int(torch.ops.replicann.gemm_get_reserve())
                                if dev.type == "cuda" and hasattr(torch.ops.replicann, "gemm_get_reserve") else None),
            "loss_first_last": [round(first_loss, 4), round(last_loss, 4)],
            **({"ce_chunk_rows": args.ce_chunk} if (is_lm and args.ce_chunk) else {}),
            **({"ddp_diag": diag} if diag is not None else {}),
            "peak_mem_gib": (round(torch.cuda.max_memory_allocated(dev) / 2**30, 2) if dev.type == "cuda" else None),
        },
    }
    if tr.rank == 0:
        if dev.type == "cuda" and os.path.isdir("gpurun_out"):  # the measured per-shape GEMM configs (runtime autotuner)
            os.makedirs("gpurun_out", exist_ok=True)
            with open(f"gpurun_out/gemm_tuning_{args.model}.json", "w") as f:
                f.write(torch.ops.replicann.gemm_tuning_table())
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
    if dist.is_initialized():
        dist.destroy_process_group()


def ddp_diagnostics(tr, world, rank_ms, sync):
    """The data-parallel step's own record (untimed, after the timed loop): device phase times of
    one eager step on every rank (``allreduce_wait_ms`` = how long the compute stream waited for the
    gradient collectives after the backward: the exposed communication), the collectives and bytes
    that step issued, the schedule the reducer actually ran (auto resolves to window / eager), the
    per-rank timed-loop ms/step spread, the RCCL version and every NCCL_* / RCCL_* setting in
    effect."""
    import torch
    import torch.distributed as dist

    comm = tr.ddp.comm
    info0 = comm.info() if hasattr(comm, "info") else None
    _, ph = tr.timed_eager_step()
    sync()
    info1 = comm.info() if hasattr(comm, "info") else None
    phases = {k: round(float(v), 3) for k, v in ph.items()}
    per_rank = [phases]
    if world > 1:
        per_rank = [None] * world
        dist.all_gather_object(per_rank, phases)
    waits = [r.get("allreduce_wait_ms") for r in per_rank if r.get("allreduce_wait_ms") is not None]
    try:
        rccl = ".".join(str(v) for v in torch.cuda.nccl.version()) if torch.cuda.is_available() else None
    except Exception:  # noqa: BLE001 - build without the nccl module
        rccl = None
    sched = tr.ddp.schedule
    if sched == "auto":
        sched = "auto->window" if getattr(tr.ddp, "_windowed", False) else "auto->eager"
    return {
        "step_phases_ms_rank0": phases,
        "allreduce_wait_ms_max": max(waits) if waits else None,
        "allreduce_wait_ms_min": min(waits) if waits else None,
        "collectives_per_step": (info1["collectives"] - info0["collectives"]) if info0 else None,
        "comm_gbytes_per_step": round((info1["bytes"] - info0["bytes"]) / 1e9, 4) if info0 else None,
        "schedule": sched,
        "reduce": ("rsag" if getattr(tr.ddp, "rsag", False) else ("fp32 all-reduce" if tr.ddp.fp32 else "bf16 all-reduce")),
        "rank_ms_per_step": rank_ms,
        "rank_ms_spread": (round(max(rank_ms) - min(rank_ms), 3) if rank_ms and None not in rank_ms else None),
        "rccl_version": rccl,
        "nccl_env": {k: v for k, v in sorted(os.environ.items()) if k.startswith(("NCCL_", "RCCL_", "TORCH_NCCL_"))},
    }


def precision(model) -> str:
    """The compute precision the timed step actually runs (not just the parameter dtype)."""
    cfg = getattr(model, "config", None)
    if getattr(cfg, "fp8", False):
        return getattr(model, "fp8_description", lambda: "fp8-e4m3 GEMMs + bf16")()
    p = next(model.parameters())
    return {"torch.bfloat16": "bf16", "torch.float32": "fp32"}.get(str(p.dtype), str(p.dtype))


if __name__ == "__main__":
    main()
