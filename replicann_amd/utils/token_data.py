"""Real-data LM input: flat binary token shards through the native loader.

The reference has no data pipeline (0 grep hits for data/IO
code); BASELINE's configs are synthetic (``utils/data.py``).  This is the path
for training GPT-2 on real tokens: ``csrc/runtime/token_loader.cpp`` (built
into ``replicann_amd/_io.so``) memory-maps the shards and fills a ring of
prefetch slots from worker threads; this wrapper copies each batch into one of
a few pinned host buffers and issues a non-blocking H2D copy, recording an
event so a pinned buffer is only rewritten after its copy has finished.

Shard format: raw little-endian uint16 (vocab < 65536, e.g. GPT-2) or uint32
tokens, no header — ``write_token_shard`` writes one.
"""

from __future__ import annotations

import ctypes
import os
from pathlib import Path
from typing import Sequence

import numpy as np
import torch

_LIB = None


def _lib():
    global _LIB
    if _LIB is None:
        from .. import _build
        # always through the hash-checked builder (cheap when up to date): a stale _io.so built
        # from older loader sources must never be dlopen'ed with the current argtypes
        path = _build.build_runtime(verbose=False)
        lib = ctypes.CDLL(str(path))
        lib.rn_loader_create.restype = ctypes.c_void_p
        lib.rn_loader_create.argtypes = [ctypes.POINTER(ctypes.c_char_p), ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                         ctypes.c_int, ctypes.c_uint64, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                         ctypes.c_int, ctypes.c_int, ctypes.c_uint64, ctypes.c_char_p, ctypes.c_int]
        lib.rn_loader_next.restype = ctypes.c_uint64
        lib.rn_loader_next.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        lib.rn_loader_num_tokens.restype = ctypes.c_uint64
        lib.rn_loader_num_tokens.argtypes = [ctypes.c_void_p]
        lib.rn_loader_num_windows.restype = ctypes.c_uint64
        lib.rn_loader_num_windows.argtypes = [ctypes.c_void_p]
        lib.rn_loader_destroy.restype = None
        lib.rn_loader_destroy.argtypes = [ctypes.c_void_p]
        _LIB = lib
    return _LIB


def write_token_shard(path, tokens, dtype=np.uint16) -> Path:
    """Write a 1-D token array as a raw shard (uint16 default, uint32 for vocab ≥ 65536)."""
    arr = np.asarray(tokens)
    if arr.size and (arr.min() < 0 or arr.max() > np.iinfo(dtype).max):
        raise ValueError(f"token ids do not fit {np.dtype(dtype).name}")
    path = Path(path)
    arr.astype(dtype).tofile(path)
    return path


class TokenFileLM:
    """Iterator of (inputs, targets) = (B, T) int64 device tensors cut from token shards.

    ``mode="train"``: random windows, a deterministic function of
    (seed, rank, batch index); ``mode="eval"``: non-overlapping windows dealt
    round-robin over ranks.  ``start_batch`` resumes the stream mid-run (the
    trainer passes ``step * grad_accum`` after a checkpoint load)."""

    def __init__(self, paths: str | Sequence[str], batch: int, seq_len: int, device, *, seed: int = 0,
                 rank: int = 0, world: int = 1, mode: str = "train", dtype: str = "uint16",
                 start_batch: int = 0, threads: int = 2, prefetch: int = 4, pinned: int = 3, vocab: int | None = None):
        if isinstance(paths, (str, os.PathLike)):
            paths = [paths]
        self.paths = [str(p) for p in paths]
        self.batch, self.seq_len, self.vocab = batch, seq_len, vocab
        self.device = torch.device(device)
        elem = {"uint16": 2, "uint32": 4}[dtype]
        arr = (ctypes.c_char_p * len(self.paths))(*[p.encode() for p in self.paths])
        err = ctypes.create_string_buffer(512)
        self._h = _lib().rn_loader_create(arr, len(self.paths), elem, batch, seq_len, seed, rank, world,
                                          {"train": 0, "eval": 1}[mode], threads, prefetch, start_batch, err, 512)
        if not self._h:
            raise ValueError(f"token loader: {err.value.decode()}")
        pin = self.device.type == "cuda"
        self._host = [torch.empty(batch, seq_len + 1, dtype=torch.int64, pin_memory=pin) for _ in range(pinned)]
        self._events = [None] * pinned
        self._i = 0
        self.batch_index = start_batch

    @property
    def num_tokens(self) -> int:
        return int(_lib().rn_loader_num_tokens(self._h))

    @property
    def num_windows(self) -> int:
        """Non-overlapping (T+1)-token windows over all shards (the eval-mode epoch length in samples)."""
        return int(_lib().rn_loader_num_windows(self._h))

    def __iter__(self):
        return self

    def __next__(self):
        slot = self._i % len(self._host)
        self._i += 1
        ev = self._events[slot]
        if ev is not None:
            ev.synchronize()  # the previous H2D copy out of this pinned buffer has finished
        buf = self._host[slot]
        self.batch_index = int(_lib().rn_loader_next(self._h, ctypes.c_void_p(buf.data_ptr()))) + 1
        if self.vocab is not None and int(buf.max()) >= self.vocab:
            raise ValueError(f"token id {int(buf.max())} >= vocab {self.vocab} in {self.paths}")
        if self.device.type == "cuda":
            t = buf.to(self.device, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
            self._events[slot] = ev
        else:
            t = buf.clone()
        return t[:, :-1], t[:, 1:]

    def state_dict(self):
        """Resume cursor (the trainer's checkpoints store it per rank)."""
        return {"batch_index": int(self.batch_index), "paths": list(self.paths)}

    def close(self):
        if getattr(self, "_h", None):
            _lib().rn_loader_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()
