"""Training / evaluation entrypoints (N21) — ``replicann.train(...)``,
``replicann.evaluate(...)`` and ``python -m replicann train|eval`` (``replicann_amd.cli``).

The reference has no training code at all; this API is
defined here and frozen.  One step:

    zero_grad (1 memset) → [fwd → loss → bwd (bucketed RCCL all-reduce
    overlapping)] × grad_accum → ddp.finish() → fused AdamW/SGD (2 kernels)

Everything inside a step is asynchronous: no host synchronisation unless a
log line needs the loss value.
"""

from __future__ import annotations

import argparse
import contextlib
import glob
import json
import time
from dataclasses import asdict, dataclass, field

import torch

from . import models
from .optim import FusedAdamW, FusedSGD, cosine_lr
from .parallel import DistributedDataParallel, init_distributed
from .utils.checkpoint import load_checkpoint, save_checkpoint
from .utils.data import SyntheticImages, SyntheticLM, SyntheticMNIST
from .utils.token_data import TokenFileLM
from .utils.flat import FlatParams
from .utils.metrics import MetricsLogger, PhaseTimer, is_rank0, phase

MODEL_KINDS = {
    "gpt2-small": "lm", "gpt2-medium": "lm", "gpt2-medium-fp8": "lm", "gpt2-tiny": "lm",
    "vit-b16": "image", "vit-tiny": "image",
    "resnet18": "image", "resnet18-tiny": "image",
    "mlp": "mnist",
    "refblock-lm": "lm",  # the reference's TransformerDecoder blocks (head dropout 0.1) as a token model
}


def build_model(name, **kw):
    if name == "gpt2-small":
        return models.GPT2(models.GPT2Config.small(**kw))
    if name == "gpt2-medium":
        return models.GPT2(models.GPT2Config.medium(**kw))
    if name == "gpt2-medium-fp8":
        return models.GPT2(models.GPT2Config.medium(fp8=True, **kw))
    if name == "gpt2-tiny":
        return models.GPT2(models.GPT2Config.tiny(**kw))
    if name == "vit-b16":
        return models.ViT(models.ViTConfig.base16(**kw))
    if name == "vit-tiny":
        return models.ViT(models.ViTConfig.tiny(**kw))
    if name == "resnet18":
        return models.ResNet18(**kw)
    if name == "resnet18-tiny":
        return models.ResNet18(num_classes=10, widths=(16, 32, 64, 128), **kw)
    if name == "mlp":
        return models.MLP(**kw)
    if name == "refblock-lm":
        return models.RefBlockLM(**kw)
    raise ValueError(f"unknown model {name!r}; known: {sorted(MODEL_KINDS)}")


@dataclass
class TrainConfig:
    model: str = "gpt2-small"
    batch_size: int = 16          # per-rank micro-batch
    seq_len: int = 1024
    image_size: int = 224
    steps: int = 20
    warmup_steps: int = 2
    lr: float = 6e-4
    min_lr_ratio: float = 0.1
    weight_decay: float = 0.1
    optimizer: str = "adamw"      # adamw | sgd
    momentum: float = 0.9
    dtype: str = "bf16"           # bf16 | fp32
    grad_accum: int = 1
    max_grad_norm: float = 1.0
    bucket_mb: float = 64.0
    # DDP cross-rank sum: rsag (default: fp32 reduce-scatter = exact sum, then a bf16 all-gather of
    # the reduced shards: 0.75x the bytes of fp32, one final rounding = the one-GPU step's gradient
    # precision) | fp32 (all-reduce in fp32, the optimizer reads it unrounded) | bf16 (in place)
    reduce_dtype: str = "rsag"
    # when a ready gradient bucket's collective is issued: auto (window once the model has shown one,
    # else eager) | eager (at once) | window (beside the next attention backward, parallel/windows.py)
    # | end (after the backward).  Measured under the 8-GPU comm proxy: profiles/ddp_window_proxy_r3ze.txt
    ddp_schedule: str = "auto"
    ddp: str = "auto"             # auto (world > 1) | on (also at world 1: one-GPU rehearsal of the DDP step)
    comm: str = "auto"            # auto (native RCCL communicator on GPUs, torch.distributed otherwise) | native | torch
    graph: str = "auto"           # auto | on | off — capture the whole step in one hipGraph
    log_every: int = 10
    metrics_path: str | None = None
    checkpoint: str | None = None
    resume: str | None = None
    # resume a checkpoint saved by another world size: model / optimizer state only, fresh per-rank
    # RNG streams and data cursors (always on for evaluation, which never uses them)
    allow_world_change: bool = False
    seed: int = 0
    device: str | None = None
    data: str | None = None       # LM token shards (comma-separated paths / globs); None = synthetic
    data_dtype: str = "uint16"    # uint16 | uint32 shard element type
    data_mode: str = "train"      # train (random windows) | eval (non-overlapping windows)
    phase_timing: bool = True     # device ms per phase (incl. comm wait) on logged eager steps
    stochastic_round: bool = True  # AdamW writes the bf16 weight copy with stochastic rounding
    model_kwargs: dict = field(default_factory=dict)


class Trainer:
    def __init__(self, cfg: TrainConfig, model=None):
        self.cfg = cfg
        self.rank, self.local_rank, self.world, dev = init_distributed(
            backend="gloo" if cfg.device == "cpu" else None, force=cfg.ddp == "on")
        self.device = torch.device(cfg.device) if cfg.device else dev
        torch.manual_seed(cfg.seed)
        if self.device.type == "cuda":
            from .ops import rng as dev_rng
            dev_rng.manual_seed(cfg.seed * 1000 + self.rank)  # device dropout streams (ops/rng.py)
        self.kind = MODEL_KINDS.get(cfg.model, "lm")
        self.model = model if model is not None else build_model(cfg.model, **cfg.model_kwargs)
        dtype = torch.bfloat16 if (cfg.dtype == "bf16" and self.device.type == "cuda") else torch.float32
        self.dtype = dtype
        self.model.to(self.device)
        for p in self.model.parameters():
            p.data = p.data.to(dtype)
        self.flat = FlatParams(self.model)
        use_ddp = self.world > 1 or cfg.ddp == "on"
        self.ddp = (DistributedDataParallel(
            self.model, self.flat, cfg.bucket_mb, comm=cfg.comm, force=True,
            reduce_dtype=torch.bfloat16 if cfg.reduce_dtype == "bf16" else torch.float32,
            reduce_mode="rsag" if cfg.reduce_dtype == "rsag" else "allreduce", schedule=cfg.ddp_schedule)
                    if use_ddp else None)
        gs = 1.0 / self.world
        if cfg.optimizer == "adamw":
            self.opt = FusedAdamW(self.flat, lr=cfg.lr, weight_decay=cfg.weight_decay,
                                  max_grad_norm=cfg.max_grad_norm, grad_scale=gs,
                                  stochastic_round=cfg.stochastic_round)
        else:
            self.opt = FusedSGD(self.flat, lr=cfg.lr, momentum=cfg.momentum, weight_decay=cfg.weight_decay,
                                max_grad_norm=cfg.max_grad_norm, grad_scale=gs)
        if self.ddp is not None:
            self.opt.grad_source = self.ddp.grad_source  # fp32 all-reduced gradients
        self.fp8_cache = None
        if self.device.type == "cuda":  # the committed per-shape GEMM configs of this model (tuning/)
            from .tuning import load_committed
            self.gemm_table_entries = load_committed(cfg.model)
        if self.device.type == "cuda":  # fp8 layers read e4m3 weights the optimizer step writes
            from .ops.fp8 import attach_weight_cache
            self.fp8_cache = attach_weight_cache(self.model, self.flat, self.opt)
        self.opt.set_schedule(cfg.warmup_steps, max(cfg.steps, 1), cfg.min_lr_ratio)
        self.step_idx = 0
        self._graph = None
        self._tuned = False
        self._resume_state = None
        if cfg.resume:
            self.step_idx, _, self._resume_state = load_checkpoint(
                cfg.resume, self.model, self.opt,
                allow_world_change=cfg.allow_world_change or cfg.data_mode != "train")
            tun = ((self._resume_state or {}).get("extra") or {}).get("gemm_tuning")
            if tun and self.device.type == "cuda":
                torch.ops.replicann.gemm_tuning_load(tun)
            if self.fp8_cache is not None:  # the saved run's e4m3 weights, same scales (no roll)
                self.fp8_cache.rebuild()
            if self.ddp is not None:
                self.ddp._broadcast_state()
        self.data = self._make_data()
        self.logger = MetricsLogger(cfg.metrics_path)
        # per-phase device times (forward / backward / allreduce_wait / optimizer) of logged eager steps
        self.timer = PhaseTimer(enabled=cfg.phase_timing)

    # ------------------------------------------------------------------
    def _make_data(self):
        c = self.cfg
        seed = c.seed * 1000 + self.rank
        saved = (self._resume_state or {}).get("data") if c.data_mode == "train" else None
        if self.kind == "lm":
            vocab = self.model.config.vocab_size
            if c.data:
                paths = sorted(p for pat in c.data.split(",") for p in (glob.glob(pat) or [pat]))
                # the stream position: the cursor saved with the checkpoint (any grad_accum), else
                # step × grad_accum for checkpoints that predate it; evaluation always starts at
                # window 0, so two checkpoints of one run are scored on the same windows
                if c.data_mode != "train":
                    start = 0
                elif saved is not None and "batch_index" in saved:
                    start = int(saved["batch_index"])
                else:
                    start = self.step_idx * c.grad_accum
                return TokenFileLM(paths, c.batch_size, c.seq_len, self.device, seed=c.seed, rank=self.rank,
                                   world=self.world, mode=c.data_mode, dtype=c.data_dtype,
                                   start_batch=start, vocab=vocab)
            src = SyntheticLM(c.batch_size, c.seq_len, vocab, self.device, seed=seed)
        elif self.kind == "image":
            m = self.model
            size = m.config.image_size if hasattr(m, "config") else c.image_size
            classes = m.config.num_classes if hasattr(m, "config") else m.fc.out_features
            src = SyntheticImages(c.batch_size, size, 3, classes, self.device, self.dtype, seed=seed)
        else:
            src = SyntheticMNIST(c.batch_size, self.device, seed=seed)
        if saved is not None:
            src.load_state_dict(saved)
        elif self.step_idx and c.data_mode == "train":
            src.load_state_dict({"i": self.step_idx * c.grad_accum})
        return src

    @property
    def net(self):
        return self.ddp if self.ddp is not None else self.model

    def samples_per_step(self):
        return self.cfg.batch_size * self.cfg.grad_accum * self.world

    def _throughput(self, steps, dt):
        """samples/s (+ tokens/s and model-FLOPs utilisation vs the bf16 dense peak for LMs)."""
        from .utils.metrics import BF16_PEAK_FLOPS
        sps = self.samples_per_step() * steps / max(dt, 1e-9)
        out = {"samples_per_s": round(sps, 2)}
        if self.kind == "lm":
            tps = sps * self.cfg.seq_len
            out["tokens_per_s"] = round(tps, 1)
            fpt = getattr(self.model, "flops_per_token", None)
            if fpt is not None:
                out["mfu"] = round(tps * fpt(self.cfg.seq_len) / (BF16_PEAK_FLOPS * self.world), 4)
        return out

    def _step_body(self, batches, lr=None):
        c = self.cfg
        self.opt.zero_grad()
        loss = None
        t = self.timer
        for micro, (x, y) in enumerate(batches):
            sync_ctx = (self.ddp.no_sync() if (self.ddp is not None and micro < len(batches) - 1)
                        else contextlib.nullcontext())
            with sync_ctx:
                with phase("forward"), t("forward"):
                    loss = self.net(x, y)
                with phase("backward"), t("backward"):
                    (loss / c.grad_accum if c.grad_accum > 1 else loss).backward()
        if self.ddp is not None:
            # device time the compute stream waits for the last all-reduces: the exposed comm
            with phase("allreduce_wait"), t("allreduce_wait"):
                self.ddp.finish()
        with phase("optimizer"), t("optimizer"):
            self.opt.step(lr)
        return loss.detach()

    def _tune(self):
        """Multi-rank GPU runs: time every GEMM shape of the step (the runtime autotuner picks
        configs on the first eager call of a shape) in one forward + backward with the reducer
        suspended, before the first real step — otherwise those timings would run beside the
        first step's RCCL all-reduces and pick configs on a busy device.  The pass is invisible
        to training: a fresh copy of the data source supplies the batch, and gradients, optimizer
        state, buffers and the device RNG streams are restored afterwards.  Multi-rank: rank 0's
        measured configs are then broadcast and adopted by every rank (one kernel choice per shape
        across the node, so the step's max-over-ranks time is not set by one rank's noisy pick)."""
        self._tuned = True
        if self.device.type != "cuda" or self.ddp is None:
            return
        from .ops import rng as dev_rng
        from .ops.fp8 import ready_restore, ready_snapshot
        probe = self._make_data()
        x, y = next(probe)
        del probe
        state = self.opt.state_tensors() + list(self.model.buffers()) + dev_rng.state_tensors(self.device)
        snap = [t.clone() for t in state]
        ready = ready_snapshot(self.model)  # fp8 delayed-scaling slots: tensors above, flags here
        with self.ddp.no_sync(), self.timer.paused():
            self.opt.zero_grad()
            self.net(x, y).backward()
        self.opt.zero_grad()
        for t, v in zip(state, snap):
            t.copy_(v)
        ready_restore(self.model, ready)
        torch.cuda.synchronize(self.device)
        if self.world > 1:  # every rank adopts rank 0's picks: the same kernels on every GPU
            import torch.distributed as dist
            box = [torch.ops.replicann.gemm_tuning_table() if self.rank == 0 else None]
            dist.broadcast_object_list(box, src=0, device=self.device if dist.get_backend() == "nccl" else None)
            if self.rank != 0:
                torch.ops.replicann.gemm_tuning_load(box[0])

    def graph_enabled(self):
        c = self.cfg
        if c.graph == "off" or self.device.type != "cuda":
            return False
        if c.graph == "on":
            return True
        # auto: single process (dropout seeds are drawn on the device — ops/rng.py — so stochastic
        # models capture too; multi-rank steps run eager: N=1 eager vs graph measured within 0.3 %,
        # profiles/graph_vs_eager_r2.txt).  A one-rank DDP rehearsal captures only with the
        # native communicator (its fork/join is capturable; torch's async works are not).
        return self.world == 1 and (self.ddp is None or self.ddp.comm.name in ("native", "proxy"))

    def _capture(self):
        """Capture zero_grad → fwd → bwd → (all-reduce) → optimizer as ONE hipGraph.

        Inputs are copied into static buffers before each replay; the LR
        schedule / bias corrections are device-side, so replays are exact.
        Two warm-up iterations run first on a side stream (they trigger the
        GEMM autotuner and every lazy allocation outside the capture); the
        training state they touch is snapshotted and restored, so graph mode
        follows exactly the same step sequence as eager mode."""
        c = self.cfg
        self._static = [tuple(t.clone() for t in next(self.data)) for _ in range(c.grad_accum)]
        from .ops import rng as dev_rng
        # fp8 delayed-scaling slots are NOT rolled back: the warm-ups seed them, so the captured step
        # is the steady-state (delayed-scaling) step, not a first step frozen into every replay
        bufs = [b for n, b in self.model.named_buffers() if not n.endswith(("fp8_scales", "fp8_gscales"))]
        state = self.opt.state_tensors() + bufs + dev_rng.state_tensors(self.device)
        snap = [t.clone() for t in state]
        count = self.opt.step_count
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s), self.timer.paused():
            for _ in range(2):
                self._step_body(self._static)
        torch.cuda.current_stream().wait_stream(s)
        for t, v in zip(state, snap):
            t.copy_(v)
        self.opt.step_count = count
        if self.fp8_cache is not None:
            self.fp8_cache.refresh()  # e4m3 weights of the restored parameters
        torch.cuda.synchronize()
        del snap
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g), self.timer.paused():
            self._static_loss = self._step_body(self._static)
        self.opt.step_count = count  # capture only recorded the step; replays count themselves
        self._graph = g
        self._static_fresh = True  # the static buffers already hold this step's batch

    def step(self, lr=None):
        """One optimizer step; returns the (device) loss of the last micro-batch.

        ``lr`` (eager mode only) overrides the device-side schedule."""
        c = self.cfg
        if not self._tuned:
            self._tune()
        if lr is None and self.graph_enabled():
            if self._graph is None:
                self._capture()
            if not self._static_fresh:
                for (sx, sy) in self._static:
                    x, y = next(self.data)
                    sx.copy_(x, non_blocking=True)
                    sy.copy_(y, non_blocking=True)
            self._static_fresh = False
            self._graph.replay()
            self.opt.step_count += 1
            self.step_idx += 1
            return self._static_loss
        batches = [next(self.data) for _ in range(c.grad_accum)]
        # phase timing only on the steps that get logged (events + one sync there)
        logged = (self.step_idx + 1) % c.log_every == 0 or self.step_idx + 1 >= c.steps
        with self.timer.step(active=logged):
            loss = self._step_body(batches, lr)
        self.step_idx += 1
        return loss

    def timed_eager_step(self):
        """One eager step with device phase timing, whatever the step form (a captured step replays
        without events): the diagnostic step bench.py records after its timed loop.  Returns
        (loss, {phase}_ms)."""
        if not self._tuned:
            self._tune()
        batches = [next(self.data) for _ in range(self.cfg.grad_accum)]
        with self.timer.step(active=True):
            loss = self._step_body(batches)
        self.step_idx += 1
        return loss, self.timer.summary()

    def save(self, path):
        """Checkpoint (collective under DDP): model, optimizer, step, config, every rank's RNG
        states and data cursor, and (GPU) the GEMM autotuner's per-shape kernel picks."""
        extra = None
        if self.device.type == "cuda":  # the GEMM kernel picks: a resumed process runs the same kernels
            extra = {"gemm_tuning": torch.ops.replicann.gemm_tuning_table()}
        save_checkpoint(path, self.model, self.opt, self.step_idx, asdict(self.cfg), extra=extra, data=self.data)

    def lr_at(self, i):
        c = self.cfg
        return cosine_lr(i, c.lr, c.warmup_steps, max(c.steps, 1), c.min_lr_ratio)

    def run(self):
        c = self.cfg
        t0 = time.time()
        start = self.step_idx
        last = None
        while self.step_idx < c.steps:
            loss = self.step()
            i = self.step_idx
            if i % c.log_every == 0 or i >= c.steps:
                lv = float(loss)
                dt = time.time() - t0
                extra = self.timer.summary()  # forward_ms, backward_ms, allreduce_wait_ms (comm wait), optimizer_ms
                if self.ddp is not None:
                    extra["comm_host_ms"] = round(self.ddp.comm_wait_ms, 3)
                    if hasattr(self.ddp.comm, "info"):  # native communicator: issued collectives / bytes
                        ci = self.ddp.comm.info()
                        extra["comm_collectives"], extra["comm_gbytes"] = ci["collectives"], round(ci["bytes"] / 1e9, 3)
                self.logger.log(step=i, loss=round(lv, 5), lr=round(float(self.opt._host_lr(None)), 8),
                                **self._throughput(i - start, dt), **extra)
                last = lv
        if c.checkpoint:
            self.save(c.checkpoint)
        return {"final_loss": last, "steps": c.steps, "wall_s": time.time() - t0}


def train(config: TrainConfig | None = None, model=None, **kw):
    """Train a replicated model; returns a summary dict.  ``model`` is an nn.Module to train, or a
    model name (same as ``TrainConfig.model``, e.g. ``train(model="gpt2-small", steps=100)``)."""
    if isinstance(model, str):
        kw["model"], model = model, None
    cfg = config or TrainConfig(**kw)
    return Trainer(cfg, model=model).run()


@torch.no_grad()
def evaluate(model, data, steps=10):
    """Mean loss (and accuracy for classifiers) over ``steps`` batches per rank; under
    data parallelism the sums are all-reduced, so every rank returns the mean over ALL
    ranks' batches (each rank reads its own round-robin share of the eval stream).

    Language models are scored through their own loss path (``model(x, targets)``: on a GPU the
    fused LM-head + cross-entropy kernels, bf16 logits consumed in place — no fp32 copy of the
    logits); classifiers through the native cross-entropy kernel."""
    from . import ops

    was = model.training
    model.eval()
    dev = next(model.parameters()).device
    sums = torch.zeros(3, dtype=torch.float64, device=dev)  # Σ loss·n, Σ correct, Σ n
    lm = _is_lm(model)
    for _ in range(steps):
        x, y = next(data)
        if lm:  # mean token loss of the batch, from the model's own fused loss path
            sums[0] += model(x, y).double() * y.numel()
            sums[2] += y.numel()
            continue
        out = model(x)
        sums[0] += ops.cross_entropy(out, y).double() * y.numel()
        sums[1] += (out.argmax(-1) == y).sum().double()
        sums[2] += y.numel()
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(sums)
    model.train(was)
    tot, cor, n = (float(v) for v in sums.cpu())
    return {"loss": tot / max(n, 1), "accuracy": cor / max(n, 1)}


def _is_lm(model) -> bool:
    """Token models (GPT-2, the reference-block LM): a vocabulary config and a targets-taking forward."""
    return hasattr(getattr(model, "config", None), "vocab_size") or hasattr(model, "vocab_size")


def eval_main(argv=None):
    """``python -m replicann eval``: mean loss (+ accuracy) of a model — random init, or a
    checkpoint written by ``train(checkpoint=...)`` — over synthetic batches, or over ``--data`` token shards in eval order."""
    ap = argparse.ArgumentParser(description="replicann evaluation entrypoint")
    ap.add_argument("--model", default="gpt2-small")
    ap.add_argument("--batch-size", type=int, default=8)
    ap.add_argument("--seq-len", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--checkpoint", default=None)
    ap.add_argument("--device", default=None)
    ap.add_argument("--model-kwargs", type=json.loads, default={})
    ap.add_argument("--data", default=None, help="LM token shards (comma-separated paths / globs)")
    ap.add_argument("--data-dtype", default="uint16")
    a = ap.parse_args(argv)
    cfg = TrainConfig(model=a.model, batch_size=a.batch_size, seq_len=a.seq_len, steps=1, device=a.device,
                      resume=a.checkpoint, model_kwargs=a.model_kwargs, graph="off", data=a.data,
                      data_dtype=a.data_dtype, data_mode="eval")
    tr = Trainer(cfg)
    out = evaluate(tr.model, tr.data, steps=a.steps)
    if is_rank0():
        print(json.dumps({"model": a.model, **out}))
    return out


def generate_main(argv=None):
    """``python -m replicann generate``: sample continuations from a GPT-2 model — random init, or a
    checkpoint written by ``train(checkpoint=...)`` — with the KV cache and the hipGraph-replayed
    decode step (``GPT2.generate``).  Prints one JSON line: the token ids, decode timing."""
    ap = argparse.ArgumentParser(description="replicann generation entrypoint (GPT-2 models)")
    ap.add_argument("--model", default="gpt2-small")
    ap.add_argument("--checkpoint", default=None)
    ap.add_argument("--prompt", default=None, help="comma-separated token ids (default: random ids)")
    ap.add_argument("--prompt-len", type=int, default=16)
    ap.add_argument("--batch-size", type=int, default=1)
    ap.add_argument("--new", type=int, default=32)
    ap.add_argument("--temperature", type=float, default=1.0)
    ap.add_argument("--top-k", type=int, default=None)
    ap.add_argument("--top-p", type=float, default=None)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--device", default=None)
    ap.add_argument("--model-kwargs", type=json.loads, default={})
    a = ap.parse_args(argv)
    if not a.model.startswith("gpt2"):
        raise SystemExit(f"generate: {a.model} is not an autoregressive GPT-2 model")
    from .utils.checkpoint import load_checkpoint
    dev = torch.device(a.device or ("cuda" if torch.cuda.is_available() else "cpu"))
    torch.manual_seed(a.seed)
    model = build_model(a.model, **a.model_kwargs)
    if a.checkpoint:
        load_checkpoint(a.checkpoint, model, restore_rng=False, allow_world_change=True)
    model = model.to(dev)
    if dev.type == "cuda":
        from .tuning import load_committed
        load_committed(a.model)
        model = model.to(torch.bfloat16)
    if a.prompt:
        ids = torch.tensor([[int(t) for t in a.prompt.split(",")]] * a.batch_size, dtype=torch.long)
    else:
        ids = torch.randint(0, model.config.vocab_size, (a.batch_size, a.prompt_len))
    gen = torch.Generator(device=dev).manual_seed(a.seed)
    t0 = time.perf_counter()
    out = model.generate(ids.to(dev), a.new, temperature=a.temperature, top_k=a.top_k, top_p=a.top_p, generator=gen)
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    res = {"model": a.model, "tokens": out[:, ids.shape[1]:].tolist(), "prompt_len": ids.shape[1],
           "new_tokens": a.new, "seconds": round(dt, 4), "tokens_per_s": round(out.shape[0] * a.new / dt, 1)}
    print(json.dumps(res))
    return res


def main(argv=None):
    ap = argparse.ArgumentParser(description="replicann_amd training entrypoint")
    for f, v in asdict(TrainConfig()).items():
        if isinstance(v, dict):
            continue
        t = type(v) if v is not None else str
        ap.add_argument(f"--{f.replace('_', '-')}", type=t, default=v)
    ap.add_argument("--model-kwargs", type=json.loads, default={})
    a = vars(ap.parse_args(argv))
    cfg = TrainConfig(**a)
    out = train(cfg)
    if is_rank0():
        print(json.dumps(out))


if __name__ == "__main__":
    main()
