"""Data parallelism: bucketed gradient all-reduce overlapped with backward — N15/N16.

One process per GPU, ``torch.distributed`` with backend ``"nccl"`` (= RCCL on
ROCm) over xGMI; ``gloo`` for the CPU tests.  The reference has no
parallelism at all; this is built MI355X-first:

* gradients are produced in ONE flat bf16 buffer (:class:`~replicann_amd.utils.flat.FlatParams`);
  the reduction runs in **fp32**: when a bucket (a contiguous slice of that buffer)
  is complete it is widened into the same slice of a flat fp32 reduction buffer and
  all-reduced there, in place — the cross-rank sum never rounds to bf16 (summing 8
  bf16 partials in a bf16 ring loses up to 3 bits).  The fused optimizer then reads
  the fp32 sums directly (``grad_source``), so there is no narrowing pass either.
  ``reduce_dtype=torch.bfloat16`` keeps the bf16-in-place variant (half the bytes);
  ``reduce_mode="rsag"`` (with fp32) splits each bucket's all-reduce into its two ring halves and
  narrows in between: an fp32 reduce-scatter (the exact cross-rank sum of this rank's shard), a
  cast of that shard to bf16, and a bf16 all-gather of the reduced shards straight into the
  gradient slice — 0.75x the wire bytes of the fp32 all-reduce, one bf16 rounding of the final
  sum (the precision a one-GPU step's bf16 gradient has), and the optimizer reads bf16 gradients.
  Buckets whose span does not split into ``world`` equal shards, and tied parameters' per-
  contribution reductions, keep the fp32 all-reduce and are narrowed in ``finish()``;
* buckets are formed in reverse parameter order (the order backward produces
  gradients) and sized for point-to-point xGMI rings (default 64 MB of reduced
  elements: large enough to amortise RCCL's per-collective latency over the 7
  links, small enough that the first bucket launches early in the backward);
* a post-accumulate-grad hook per parameter (and ``FlatParams.mark_ready`` for the
  gradients kernels accumulate directly) counts arrivals; a complete bucket's
  ``all_reduce(SUM, async_op=True)`` is issued at once — RCCL runs it on its own HIP
  stream, ordered after the producing kernels, overlapping the rest of the backward;
* **tied parameters are split**: a parameter with several direct gradient
  contributions per backward (GPT-2's ``wte``: LM-head weight gradient at the START
  of the backward, embedding scatter at the END) gets a bucket of its own, and EACH
  contribution is reduced as soon as it exists — the first one into the reduction
  buffer, later ones into side buffers that ``finish()`` adds in (the bf16 slice is
  cleared between contributions).  Without the split the 38.6 M-element ``wte``
  bucket waited for the embedding backward and ran fully exposed after it;
* buckets are LAUNCHED in index order (a ready bucket waits for its predecessors) and
  split contributions at their (deterministic) arrival, so every rank issues the same
  collective sequence;
* the 1/world averaging is NOT a separate pass: it is folded into the fused
  optimizer's ``grad_scale``;
* ``finish()`` waits on the outstanding works (stream-ordered, no host sync),
  launches buckets whose parameters received no gradient (unused parameters:
  their slice is zero on every rank), and checks every bucket was reduced
  exactly once;
* **when** a ready bucket's collective is issued (``schedule``; ``"auto"``, the default, is
  ``"window"`` once a step has shown a window and ``"eager"`` otherwise): ``"eager"`` at once (the classic
  overlap), ``"window"`` queued until the next communication window — the attention backward, whose
  short workgroups a high-priority collective interleaves with (``parallel/windows.py``) — at most
  ``window_mb`` of reduction bytes per window (a larger tied-parameter contribution is split into
  pieces), the rest in ``finish()``; ``"end"`` everything in ``finish()``.  The widening copy always
  runs when the bucket is ready.  Why not simply eager: the persistent GEMM owns every CU, and a
  collective beside it delays the GEMM's workgroups on the CUs it holds for its whole duration
  (profiles/ddp_window_proxy_r3ze.txt);
* ``no_sync()`` disables reduction for gradient accumulation;
* construction broadcasts rank 0's parameters and buffers (one flat broadcast);
* the collectives go through a :mod:`~replicann_amd.parallel.comm` back-end: on GPUs
  over an ``nccl`` group the framework's own RCCL communicator (``csrc/comm``: a
  high-priority comm stream forked/joined by events — hipGraph-capturable — plus a
  hang/async-error watchdog), otherwise ``torch.distributed`` async works (gloo tests);
* ``force=True`` keeps the reducer active at world size 1 (a one-GPU rehearsal of the
  multi-GPU step: same widening copies, same collective calls, same stream joins).
"""

from __future__ import annotations

import contextlib
import time

import torch
import torch.distributed as dist
import torch.nn as nn

from ..utils.flat import FlatParams
from .comm import make_comm


class DistributedDataParallel(nn.Module):
    def __init__(self, module: nn.Module, flat: FlatParams, bucket_mb: float = 64.0,
                 process_group=None, broadcast: bool = True, check_unused: bool = False,
                 reduce_dtype=torch.float32, split_tied: bool = True, comm="auto", force: bool = False,
                 reduce_mode: str = "allreduce", schedule: str = "auto", window_mb: float | None = None):
        super().__init__()
        self.module = module
        self.flat = flat
        self.pg = process_group
        self.world = dist.get_world_size(process_group) if dist.is_initialized() else 1
        self.active = self.world > 1 or force  # reduce at all (force: one-rank rehearsal)
        self.check_unused = check_unused
        self._sync = True
        self.comm = make_comm(comm, process_group, flat.grad.device) if isinstance(comm, str) else comm
        self._reserve_cus()
        if broadcast and self.world > 1:
            self._broadcast_state()
        self.reduce_dtype = reduce_dtype
        self.fp32 = reduce_dtype == torch.float32 and flat.grad.dtype != torch.float32
        # the buffer the all-reduce runs on (and the optimizer reads): fp32 copy, or the grads themselves
        self.reduce_buf = (torch.zeros(flat.numel, dtype=torch.float32, device=flat.grad.device)
                           if self.fp32 else flat.grad)
        if reduce_mode not in ("allreduce", "rsag"):
            raise ValueError(f"reduce_mode {reduce_mode!r}: allreduce | rsag")
        # rsag: fp32 reduce-scatter + bf16 all-gather (needs the fp32 reduction of bf16 gradients)
        self.rsag = reduce_mode == "rsag" and self.fp32 and flat.grad.dtype == torch.bfloat16
        if self.rsag:  # shard scratch: bucket [lo, hi) owns [lo / world, hi / world)
            W = self.world
            self.rs32 = torch.zeros(flat.numel // W + 1, dtype=torch.float32, device=flat.grad.device)
            self.rs16 = torch.zeros(flat.numel // W + 1, dtype=torch.bfloat16, device=flat.grad.device)
        self.tie_rs = {}  # rsag: tied parameter -> one fp32 shard per contribution (summed in finish)
        self._narrow = []  # fp32-reduced spans to narrow into the bf16 gradient in finish() (rsag)
        if schedule not in ("auto", "eager", "window", "end"):
            raise ValueError(f"schedule {schedule!r}: auto | eager | window | end")
        self.schedule = schedule
        # auto: eager until a step has shown a window (a model without attention backward keeps
        # eager), window from the next step on — every rank runs the same model, so the switch is
        # at the same step everywhere
        self._windowed = schedule == "window"
        self._saw_window = False
        if window_mb is None:  # REPLICANN_DDP_WINDOW_MB: reduction bytes issued per window (default 64)
            import os
            window_mb = float(os.environ.get("REPLICANN_DDP_WINDOW_MB", 64.0))
        self.window_bytes = int(window_mb * 1024 * 1024)
        self._queue = []  # prepared collectives waiting for a window (schedule window / end)
        if schedule in ("window", "auto"):
            from .windows import register
            register(self._window)
        # ---- bucket assignment (reverse layout order); split (tied) parameters alone ----
        segs = flat.segments()
        self.split = {}  # id(p) -> [lo, hi, uses, side buffers]
        if split_tied:
            for p, off, n in segs:
                uses = getattr(p, "_rn_direct_uses", 1)
                if uses > 1 and flat.direct:
                    sides = [torch.zeros(n, dtype=self.reduce_buf.dtype, device=flat.grad.device)
                             for _ in range(uses - 1)]
                    self.split[id(p)] = [off, off + n, uses, sides]
        elem = self.reduce_buf.element_size()
        cap = max(1, int(bucket_mb * 1024 * 1024 / elem))
        self.buckets = []  # (lo, hi, n_params)
        self.param_bucket = {}
        cur_hi = None
        cur_lo = None
        cur_n = 0
        for p, off, n in reversed(segs):
            if id(p) in self.split:
                continue
            end = flat.span(p)[1]
            if cur_hi is None:
                cur_hi, cur_lo, cur_n = end, off, 0
            elif (cur_hi - off > cap or cur_lo != end) and cur_n > 0:
                # a split parameter between two neighbours breaks contiguity: close the bucket
                self.buckets.append([cur_lo, cur_hi, cur_n])
                cur_hi, cur_lo, cur_n = end, off, 0
            cur_lo = off
            cur_n += 1
            self.param_bucket[id(p)] = len(self.buckets)
        if cur_hi is not None:
            self.buckets.append([cur_lo, cur_hi, cur_n])
        self._split_params = {id(p): p for p, _, _ in segs if id(p) in self.split}
        if self.rsag:
            for pid, (lo, hi, uses, _) in self.split.items():
                if (hi - lo) % self.world == 0 and lo % self.world == 0:
                    self.tie_rs[pid] = [torch.zeros((hi - lo) // self.world, dtype=torch.float32,
                                                    device=flat.grad.device) for _ in range(uses)]
        self._reset()
        self._hooks = [p.register_post_accumulate_grad_hook(self._hook) for p, _, _ in segs]
        flat.ready_hooks.append(self._hook)  # parameters whose grads are accumulated directly by kernels
        flat.contribution_hooks.append(self._contribution)
        self.comm_wait_ms = 0.0  # host time spent in finish() (last step): the exposed all-reduce tail

    _sched_ops = None  # set in "overlap" schedule mode

    def _reserve_cus(self):
        """GEMM schedule knobs for steps whose collectives run beside the backward (world > 1,
        or the one-GPU comm proxy).  ``REPLICANN_GEMM_SCHED=dynamic`` makes the persistent GEMM
        dequeue its tiles (csrc/include/gemm_pk.h, "Tile schedule"): a workgroup that starts
        late because RCCL holds its CU takes fewer tiles instead of stalling the whole GEMM.
        It is opt-in: on GPT-2-small under the proxy the queue's per-K-tile atomic costs more
        than it recovers (68.2 ms static vs 70.6 ms dynamic per step, profiles/
        gemm_sched_proxy_r3f.txt).  ``REPLICANN_GEMM_RESERVE`` CUs (default 0) can additionally
        be left free for the collectives' workgroups (measured: a reservation costs more in
        wave quantisation than it saves, profiles/gemm_sched_ab_r3d.txt)."""
        import os

        dev = self.flat.grad.device
        if dev.type != "cuda" or not (self.world > 1 or getattr(self.comm, "proxy", False)):
            return
        from .. import _ext

        ops = _ext.ops()
        mode = os.environ.get("REPLICANN_GEMM_SCHED", "static")
        if mode == "dynamic":
            ops.gemm_set_sched(1)
        elif mode == "overlap":  # queue only for the GEMMs launched while a collective is in flight
            ops.gemm_sched_init(dev.index if dev.index is not None else torch.cuda.current_device())
            self._sched_ops = ops
        ops.gemm_set_reserve(int(os.environ.get("REPLICANN_GEMM_RESERVE", 0)))
        self.gemm_reserve = ops.gemm_get_reserve()
        self.gemm_sched = ops.gemm_get_sched()

    # ------------------------------------------------------------------
    def _broadcast_state(self):
        self.comm.broadcast(self.flat.data, 0)
        for b in self.module.buffers():
            if b.is_contiguous() and b.numel():
                self.comm.broadcast(b.data, 0)
        self.comm.wait()

    def _reset(self):
        self._narrow = []
        self._queue = []
        self._tie_plan = {}  # tied parameter -> the reduce-scatter pieces this step (rsag)
        self._pending = [b[2] for b in self.buckets]
        self._ready = [False] * len(self.buckets)
        self._launched = [False] * len(self.buckets)
        self._next = 0
        self._seen = set()
        self._split_done = {k: 0 for k in self.split}  # contributions reduced this step
        self.launched_in_backward = 0

    def _reduce_slice(self, lo, hi, dst=None, whole=True):
        """Prepare (widen, now) and issue or queue (``schedule``) the reduction of grad[lo:hi]."""
        for job in self._prepare(lo, hi, dst, whole):
            self._submit(job)

    def _submit(self, job):
        if self.schedule == "eager" or (self.schedule == "auto" and not self._windowed):
            self._issue(job)
        else:
            self._queue.append(job)

    def _job_bytes(self, job):
        if job[0] == "rsag":
            return (job[2] - job[1]) * 4
        return job[1].numel() * job[1].element_size()  # "ar" (buffer) / "rs" (input)

    def _tie_chunks(self, n):
        """[start, end) pieces of a tied span of n elements: each a multiple of world (the reduce-
        scatter and the final all-gather use the same pieces, so the shard layout matches)."""
        W = self.world
        if not self._windowed and self.schedule != "end":
            return [(0, n)]
        m = max(W, (self.window_bytes // 4) // W * W)
        return [(i, min(i + m, n)) for i in range(0, n, m)]

    def _tie_contribution(self, pid, k):
        """rsag, tied parameter: widen contribution k (the slice's current content) and reduce-scatter
        it, piece by piece, into its fp32 shard (the shards are summed and all-gathered in finish())."""
        lo, hi, uses, sides = self.split[pid]
        src = self.reduce_buf[lo:hi] if k == 0 else sides[k - 1]
        src.copy_(self.flat.grad[lo:hi])
        W, sh = self.world, self.tie_rs[pid][k]
        # the pieces are fixed by the step's first contribution: every contribution's shard and the
        # final all-gather must share one layout even if the schedule changes at finish() (auto)
        plan = self._tie_plan.setdefault(pid, self._tie_chunks(hi - lo))
        for a, b in plan:
            self._submit(("rs", src[a:b], sh[a // W:b // W]))

    def _issue(self, job):
        if job[0] == "rsag":
            _, lo, hi = job
            W = self.world
            o, n = lo // W, (hi - lo) // W
            self.comm.reduce_scatter(self.reduce_buf[lo:hi], self.rs32[o:o + n])
            self.comm.narrow_all_gather(self.rs32[o:o + n], self.rs16[o:o + n], self.flat.grad[lo:hi])
        elif job[0] == "rs":
            self.comm.reduce_scatter(job[1], job[2])
        else:
            self.comm.all_reduce(job[1])
        if self._sched_ops is not None:
            self._sched_ops.gemm_set_sched(1)  # later GEMMs of this backward share the CUs with RCCL

    def _window(self):
        """A communication window opened: issue queued collectives, up to ``window_bytes``."""
        if not (self._sync and self.active):
            return
        self._saw_window = True
        if not self._windowed or not self._queue:
            return
        used = 0
        while self._queue and (used == 0 or used + self._job_bytes(self._queue[0]) <= self.window_bytes):
            job = self._queue.pop(0)
            used += self._job_bytes(job)
            self._issue(job)

    def _prepare(self, lo, hi, dst=None, whole=True):
        """Widen (fp32 mode) and all-reduce grad[lo:hi]; ``dst`` overrides the target buffer.
        rsag mode: a whole bucket that splits into ``world`` equal shards is reduce-scattered in fp32
        and all-gathered back into grad[lo:hi] in bf16 instead (``whole`` False: one contribution of a
        split parameter, summed with the others in fp32 in finish(): always the fp32 all-reduce)."""
        g = self.flat.grad[lo:hi]
        W = self.world
        if self.rsag and whole and dst is None and (hi - lo) % W == 0 and lo % W == 0:
            self.reduce_buf[lo:hi].copy_(g)  # widen: the reduce-scatter sums in fp32
            return [("rsag", lo, hi)]
        if dst is None:
            dst = self.reduce_buf[lo:hi]
        if self.rsag:
            self._narrow.append((lo, hi))
        if dst.data_ptr() != g.data_ptr():
            dst.copy_(g)  # stream-ordered after the kernels that produced the gradient
        if not self._windowed and self.schedule != "end":
            return [("ar", dst)]
        # queued: pieces of at most one window's budget (a tied contribution can exceed it)
        step = max(1, self.window_bytes // dst.element_size())
        return [("ar", dst[i:i + step]) for i in range(0, dst.numel(), step)]

    def _launch_ready(self, from_hook=False):
        while self._next < len(self.buckets) and self._ready[self._next]:
            self.launched_in_backward += int(from_hook)
            lo, hi, _ = self.buckets[self._next]
            self._reduce_slice(lo, hi)
            self._launched[self._next] = True
            self._next += 1

    def _contribution(self, p, final):
        """A direct gradient contribution to a split parameter is complete (``final``: its last)."""
        if not self._sync or not self.active or id(p) not in self.split:
            return
        lo, hi, uses, sides = self.split[id(p)]
        k = self._split_done[id(p)]
        if k >= uses:
            return
        g = self.flat.grad[lo:hi]
        if id(p) in self.tie_rs:  # rsag: reduce-scatter now, one bf16 all-gather of the summed shards later
            self._tie_contribution(id(p), k)
            if not final:
                g.zero_()
        elif self.fp32:
            # contribution 0 → the reduction buffer, later ones → side buffers (added in finish)
            self._reduce_slice(lo, hi, None if k == 0 else sides[k - 1], whole=False)
            if not final:
                g.zero_()  # the next contribution accumulates into a cleared slice
        elif final:
            self._reduce_slice(lo, hi)  # bf16 in place: only this contribution is left in the slice
        else:
            sides[k].copy_(g)
            g.zero_()
            self.comm.all_reduce(sides[k])
        self._split_done[id(p)] = k + 1
        self.launched_in_backward += 1

    def _hook(self, p):
        if not self._sync or not self.active:
            return
        if id(p) in self.split:
            return  # handled per contribution
        if id(p) in self._seen:  # a parameter used twice accumulates twice: count once
            return
        self._seen.add(id(p))
        bi = self.param_bucket[id(p)]
        self._pending[bi] -= 1
        if self._pending[bi] == 0:
            self._ready[bi] = True
            self._launch_ready(from_hook=True)

    # ------------------------------------------------------------------
    def forward(self, *args, **kwargs):
        if self._sync:
            self._reset()
        return self.module(*args, **kwargs)

    @property
    def grad_source(self):
        """The tensor holding the all-reduced (SUM over ranks) flat gradient after ``finish()``:
        the fp32 reduction buffer, or (rsag) the bf16 gradient buffer itself."""
        return self.flat.grad if self.rsag else self.reduce_buf

    reduced_grad = grad_source

    def finish(self):
        """Complete the gradient reduction (call after backward, before the optimizer)."""
        if not self._sync or not self.active:
            return
        t0 = time.perf_counter()
        unused = [i for i, r in enumerate(self._ready) if not r]
        if unused and self.check_unused:
            names = [self.flat.names.get(id(p), "?") for p, _, _ in self.flat.segments()
                     if id(p) not in self._seen and id(p) not in self.split]
            raise RuntimeError(f"parameters received no gradient this step: {names[:8]}")
        for i in unused:
            self._ready[i] = True
        self._launch_ready()
        # split parameters: contributions that never arrived (e.g. autograd-accumulated on CPU,
        # where both uses land in .grad at once) are reduced now, as one
        for pid, (lo, hi, uses, sides) in self.split.items():
            k = self._split_done[pid]
            if k < uses and pid in self.tie_rs:
                self._tie_contribution(pid, k)  # the slice holds every missing contribution: as one
                for sh in self.tie_rs[pid][k + 1:]:
                    sh.zero_()
            elif k < uses:
                # the contributions that never signalled (e.g. autograd accumulated both uses at
                # once, CPU path) are all in the slice: reduce it as ONE contribution
                if self.fp32 and k > 0:
                    self._reduce_slice(lo, hi, sides[k - 1], whole=False)
                    unused_sides = sides[k:]
                else:
                    # fp32: contribution 0; bf16: in place, sides[:k] hold the rest
                    self._reduce_slice(lo, hi, whole=False)
                    unused_sides = sides[k:]
                for s_ in unused_sides:
                    s_.zero_()
            self._split_done[pid] = uses
        while self._queue:  # collectives no window took (schedule window / end), in queue order
            self._issue(self._queue.pop(0))
        if self.schedule == "auto":
            self._windowed = self._saw_window
        self.comm.wait()  # native: the compute stream joins the comm stream (no host sync)
        if self._sched_ops is not None:
            self._sched_ops.gemm_set_sched(0)
        for pid, (lo, hi, uses, sides) in self.split.items():
            if pid in self.tie_rs:  # rsag: sum the contributions' fp32 shards, narrow, bf16 all-gather
                sh = self.tie_rs[pid]
                for extra in sh[1:]:
                    sh[0].add_(extra)
                W = self.world
                for a, b in self._tie_plan[pid]:
                    self.comm.narrow_all_gather(sh[0][a // W:b // W], self.rs16[(lo + a) // W:(lo + b) // W],
                                                self.flat.grad[lo + a:lo + b], after_rs=False)
                continue
            for s in sides:
                self.reduce_buf[lo:hi].add_(s)
        if self.tie_rs:
            self.comm.wait()
        # rsag: spans that took the fp32 all-reduce (tied contributions, unevenly split buckets) are
        # narrowed into the bf16 gradient the optimizer reads
        for lo, hi in dict.fromkeys(self._narrow):
            self.flat.grad[lo:hi].copy_(self.reduce_buf[lo:hi])
        assert all(self._launched), "a gradient bucket was never reduced"
        self.comm_wait_ms = (time.perf_counter() - t0) * 1e3

    @contextlib.contextmanager
    def no_sync(self):
        prev = self._sync
        self._sync = False
        try:
            yield
        finally:
            self._sync = prev

    @property
    def grad_scale(self):
        return 1.0 / self.world
