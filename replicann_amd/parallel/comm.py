"""Collective back-ends for the data-parallel reducer (SURVEY.md §1 L1', N16).

Two implementations of one small interface (``all_reduce`` / ``broadcast`` /
``all_gather`` / ``reduce_scatter`` / ``narrow_all_gather`` issue asynchronously, ``wait`` joins
them into the caller's stream, ``synchronize`` blocks the host):

* :class:`NativeComm` — the framework's own RCCL communicator
  (``csrc/comm/rccl_comm.cpp``): collectives on a dedicated high-priority HIP comm
  stream forked from the compute stream by an event, a watchdog thread that aborts a
  hung or failed communicator, and hipGraph-capturable fork/join.  The ncclUniqueId is
  drawn by rank 0 and exchanged over the ``torch.distributed`` rendezvous;
* :class:`TorchComm` — ``torch.distributed`` async collectives (``nccl`` = RCCL on a
  GPU, ``gloo`` on the CPU).  The CPU tests and gloo rehearsals run this one.

``make_comm("auto")`` picks native for a ONE-rank ``nccl`` group (the one-GPU rehearsal,
where it is hardware-tested and hipGraph-capturable) and torch otherwise: at world > 1 the
native communicator has not yet been run on a multi-GPU node, so ProcessGroupNCCL (also RCCL,
on its own internal stream) stays the default there until a multi-GPU parity run of the native
path exists; ``REPLICANN_COMM=native`` (or ``comm="native"``) opts in.  The reference has no collective code (``/root/reference/poetry.lock:1222``
is its only NCCL touchpoint).
"""

from __future__ import annotations

import os

import torch
import torch.distributed as dist

_OPS = {"sum": 0, "max": 1, "min": 2, "avg": 3}


class TorchComm:
    """``torch.distributed`` async collectives; ``wait`` waits on the outstanding works."""

    name = "torch"

    def __init__(self, group=None):
        self.group = group
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self._works = []
        self._n = 0  # collectives issued and bytes handed to them (this rank's buffer; info())
        self._bytes = 0

    def _count(self, t):
        self._n += 1
        self._bytes += t.numel() * t.element_size()

    def info(self):
        """Issued collectives and their bytes so far (same keys as the native communicator's)."""
        return {"rank": self.rank, "world": self.world, "collectives": self._n, "bytes": self._bytes, "failed": False}

    def all_reduce(self, t, op="sum"):
        rop = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN}[op]
        self._count(t)
        self._works.append(dist.all_reduce(t, op=rop, group=self.group, async_op=True))

    def broadcast(self, t, root=0):
        self._count(t)
        self._works.append(dist.broadcast(t, root, group=self.group, async_op=True))

    def all_gather(self, inp, out):
        self._count(out)
        self._works.append(dist.all_gather_into_tensor(out, inp, group=self.group, async_op=True))

    def reduce_scatter(self, inp, out, op="sum"):
        self._count(inp)
        self._works.append(dist.reduce_scatter_tensor(out, inp, group=self.group, async_op=True))

    _side = None

    def narrow_all_gather(self, shard32, shard16, full, after_rs=True):
        """After ``reduce_scatter(…, shard32)``: narrow this rank's reduced fp32 shard into ``shard16``
        and all-gather the bf16 shards into ``full`` — on a side stream that waits for the
        reduce-scatter, so the compute stream is not held (GPU); in order on the CPU.
        ``after_rs=False``: shard32 was produced on the current stream instead (e.g. a sum of shards)."""
        rs = self._works[-1] if after_rs else None
        if shard32.is_cuda:
            if self._side is None:
                self._side = torch.cuda.Stream(device=shard32.device)
            cur = torch.cuda.current_stream(shard32.device)
            with torch.cuda.stream(self._side):
                if rs is not None:
                    rs.wait()  # the side stream waits for the reduce-scatter's completion
                else:
                    self._side.wait_stream(cur)
                shard16.copy_(shard32)
                # issued from the side stream: the collective is ordered after the narrowing copy
                self._count(full)
                self._works.append(dist.all_gather_into_tensor(full, shard16, group=self.group, async_op=True))
        else:
            if rs is not None:
                rs.wait()
            shard16.copy_(shard32)
            self._count(full)
            self._works.append(dist.all_gather_into_tensor(full, shard16, group=self.group, async_op=True))

    def wait(self):
        for w in self._works:
            w.wait()
        self._works = []

    synchronize = wait

    def close(self):
        self.wait()


class NativeComm:
    """The framework's RCCL communicator (``torch.ops.replicann.comm_*``) for one device.

    Lifetime contract: a tensor handed to a collective must stay alive (not be freed / reused)
    until :meth:`wait` has joined the comm stream into the stream that frees it — the DDP reducer's
    buckets are persistent slices of its flat buffers.  (Registering the comm stream with the
    caching allocator via recordStream on the external stream crashed in round-2 testing.)"""

    name = "native"

    def __init__(self, group=None, device=None, timeout_s: float = 600.0, proxy: bool = False):
        from .. import _ext

        self.ops = _ext.ops()
        self.group = group
        if dist.is_initialized():
            self.rank, self.world = dist.get_rank(group), dist.get_world_size(group)
        else:
            self.rank, self.world = 0, 1
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.proxy = proxy
        if proxy:
            # one-GPU stand-in for an N-GPU RCCL collective's footprint (csrc/kernels/comm_proxy.hip):
            # REPLICANN_PROXY_WORLD emulated ranks, REPLICANN_PROXY_WGS workgroups, REPLICANN_PROXY_GBPS
            # per-GPU bus bandwidth of the emulated xGMI ring
            assert self.world == 1, "the comm proxy stands in for collectives on a one-rank group"
            self.name = "proxy"
            self.proxy_world = int(os.environ.get("REPLICANN_PROXY_WORLD", 8))
            self.proxy_wgs = int(os.environ.get("REPLICANN_PROXY_WGS", 32))
            self.proxy_gbps = float(os.environ.get("REPLICANN_PROXY_GBPS", 300.0))
            self.handle = int(self.ops.comm_init_proxy(self.device.index, self.proxy_world, self.proxy_wgs,
                                                       self.proxy_gbps, float(timeout_s)))
            import atexit

            atexit.register(self._quiesce)
            return
        uid = self.ops.comm_unique_id() if self.rank == 0 else None
        if self.world > 1:  # rank 0's id over the existing rendezvous (a CPU object broadcast)
            box = [bytes(uid.numpy()) if uid is not None else None]
            dist.broadcast_object_list(box, src=dist.get_global_rank(group, 0) if group is not None else 0,
                                       group=group, device=self.device if _is_nccl(group) else None)
            uid = torch.frombuffer(bytearray(box[0]), dtype=torch.uint8)
        self.handle = int(self.ops.comm_init(uid, self.rank, self.world, self.device.index, float(timeout_s)))
        import atexit

        atexit.register(self._quiesce)  # watchdog stopped before the HIP runtime tears down

    def _quiesce(self):
        if self.handle is not None:
            self.ops.comm_quiesce(self.handle)

    def all_reduce(self, t, op="sum"):
        self.ops.comm_all_reduce(self.handle, t, _OPS[op])

    def broadcast(self, t, root=0):
        self.ops.comm_broadcast(self.handle, t, root)

    def all_gather(self, inp, out):
        self.ops.comm_all_gather(self.handle, inp, out)

    def reduce_scatter(self, inp, out, op="sum"):
        self.ops.comm_reduce_scatter(self.handle, inp, out, _OPS[op])

    def narrow_all_gather(self, shard32, shard16, full, after_rs=True):
        """Narrow + bf16 all-gather on the comm stream, after the preceding reduce-scatter (and, being
        forked from the current stream, after whatever produced shard32 there)."""
        self.ops.comm_narrow_all_gather(self.handle, shard32, shard16, full)

    def wait(self):
        """The current stream waits for every collective issued so far (stream-ordered)."""
        self.ops.comm_wait(self.handle)

    def synchronize(self):
        self.ops.comm_synchronize(self.handle)

    def info(self):
        r, w, n, b, failed = self.ops.comm_info(self.handle)
        return {"rank": r, "world": w, "collectives": n, "bytes": b, "failed": bool(failed)}

    def close(self):
        if self.handle is not None:
            self.ops.comm_destroy(self.handle)
            self.handle = None


def _is_nccl(group=None) -> bool:
    return dist.is_initialized() and dist.get_backend(group) == "nccl"


def make_comm(kind: str = "auto", group=None, device=None, timeout_s: float = 600.0):
    """``kind``: ``auto`` (env ``REPLICANN_COMM`` if set; else native on an nccl group),
    ``native`` or ``torch``.  ``REPLICANN_COMM_TIMEOUT`` overrides ``timeout_s``."""
    if kind == "auto":
        kind = os.environ.get("REPLICANN_COMM", "auto")
    # REPLICANN_COMM_TIMEOUT (seconds): the native watchdog's hang limit per collective
    timeout_s = float(os.environ.get("REPLICANN_COMM_TIMEOUT", timeout_s))
    dev = torch.device(device) if device is not None else None
    if kind == "auto":
        world = dist.get_world_size(group) if dist.is_initialized() else 1
        if _is_nccl(group) and world == 1 and (dev is None or dev.type == "cuda"):
            try:
                return NativeComm(group, dev, timeout_s)
            except Exception as e:  # e.g. extension built without RCCL: same collectives via torch
                import warnings

                warnings.warn(f"native RCCL communicator unavailable ({e}); using torch.distributed")
                return TorchComm(group)
        kind = "torch"
    if kind == "native":
        return NativeComm(group, dev, timeout_s)
    if kind == "proxy":
        return NativeComm(group, dev, timeout_s, proxy=True)
    if kind == "torch":
        return TorchComm(group)
    raise ValueError(f"unknown comm kind {kind!r} (auto | native | torch | proxy)")
