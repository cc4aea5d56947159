"""In-tree native build for the gfx950 extension ``replicann_amd/_C.so``.

There is no native code in the reference; this is the N1
component: every ``csrc/kernels/*.hip`` is compiled by ``hipcc
--offload-arch=gfx950`` as a plain HIP translation unit (no torch headers, so
they build in seconds), ``csrc/bindings/*.cpp`` register the ops with the
PyTorch dispatcher (``TORCH_LIBRARY(replicann, ...)``), and everything is
linked into one shared object next to this file.  The ``.so`` travels with the
repo snapshot to the GPU box (it is git-ignored, not gpurun-ignored).

Rebuilds are incremental: each object is keyed by a hash of its source, the
shared headers and the flags.
"""

from __future__ import annotations

import contextlib
import fcntl
import hashlib
import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
CSRC = ROOT / "csrc"
BUILD = ROOT / "build" / "objs"
# REPLICANN_BUILD_OUT: write the library elsewhere (developer A/B builds, e.g. REPLICANN_DEV=1 ablations
# loaded with REPLICANN_SO), leaving the tree's production _C.so untouched
OUT = Path(os.environ.get("REPLICANN_BUILD_OUT") or Path(__file__).resolve().parent / "_C.so")
ARCH = os.environ.get("REPLICANN_ARCH", "gfx950")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")

HIP_FLAGS = [
    f"--offload-arch={ARCH}",
    "-O3",
    "-fPIC",
    "-std=c++17",
    "-ffp-contract=fast",
    "-munsafe-fp-atomics",
    "-Wno-unused-result",
]
if os.environ.get("REPLICANN_CHECK", "0") == "1":  # debug build: device bounds checks (RN_CHECK)
    HIP_FLAGS.append("-DREPLICANN_CHECK=1")
# developer build: also links the timing-only GEMM ablation kernels (gemm_pk_dbg.hip, cfg 90+:
# WRONG outputs by design), which a default build neither compiles nor dispatches to
DEV = os.environ.get("REPLICANN_DEV", "0") == "1"
if DEV:
    HIP_FLAGS.append("-DREPLICANN_DEV=1")
DEV_ONLY = {"gemm_pk_dbg"}
# A/B experiments: extra preprocessor definitions (space-separated NAME[=VALUE]), dev builds only
if DEV:
    HIP_FLAGS += [f"-D{d}" for d in os.environ.get("REPLICANN_EXTRA_DEFS", "").split()]

# Per-translation-unit extra flags.  The attention kernels run VALU-bound beside their MFMAs;
# SLP vectorisation packs adjacent f32 adds/muls into v_pk_add/v_pk_mul_f32, which cost ~22-26
# extra cycles each next to an MFMA (MI355X guide: 'price of one filler beside MFMAs').
FILE_FLAGS = {
    "attention": os.environ.get("REPLICANN_ATTN_FLAGS", "-fno-slp-vectorize").split(),
}


def _torch_paths():
    import torch

    tdir = Path(torch.__file__).resolve().parent
    inc = [tdir / "include", tdir / "include" / "torch" / "csrc" / "api" / "include"]
    lib = tdir / "lib"
    return inc, lib


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found: the gfx950 extension cannot be built")


def _headers_digest() -> str:
    h = hashlib.sha1()
    for p in sorted((CSRC / "include").glob("*.h")):
        h.update(p.read_bytes())
    return h.hexdigest()


def _compile(src: Path, hdr: str, torch_inc) -> Path:
    is_binding = src.suffix == ".cpp"
    flags = list(HIP_FLAGS) + FILE_FLAGS.get(src.stem, []) + [f"-I{CSRC / 'include'}"]
    if is_binding:
        # host-only TU: torch headers, no device code
        flags = [f for f in flags if not f.startswith("--offload-arch")]
        flags += ["-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1", "-O2", "--offload-host-only"]
        flags += [f"-I{p}" for p in torch_inc]
    key = hashlib.sha1((src.read_text() + hdr + " ".join(flags)).encode()).hexdigest()[:16]
    obj = BUILD / f"{src.stem}.{key}.o"
    if obj.exists():
        return obj
    tmp = f"{obj}.tmp.{os.getpid()}"
    cmd = [_hipcc()] + flags + ["-c", str(src), "-o", tmp]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src.name}:\n{r.stderr[-6000:]}")
    os.replace(tmp, obj)
    return obj


IO_OUT = Path(__file__).resolve().parent / "_io.so"
SRC_STAMP = OUT.with_suffix(".srcstamp")


def _sources():
    """Every source that goes into ``_C.so`` (the dev-only ablation kernels only in a dev build)."""
    return [s for s in (sorted((CSRC / "kernels").glob("*.hip")) + sorted((CSRC / "bindings").glob("*.cpp"))
                        + sorted((CSRC / "comm").glob("*.cpp"))) if DEV or s.stem not in DEV_ONLY]


def source_digest() -> str:
    """Location-independent digest of what ``_C.so`` is built from: the relative path and bytes
    of every compiled source and shared header.  Written next to the library at link time (first
    line of ``_C.srcstamp``); ``_ext.load()`` recomputes it and refuses a library built from other
    sources (a stale ``_C.so`` pushed with a newer tree).  The build-mode ``-D`` flags are recorded
    on the stamp's second line (``build_defs()``) instead of being folded in here: they describe
    the build, and a process whose environment differs from the build's must still load it."""
    h = hashlib.sha1()
    for p in sorted(_sources() + sorted((CSRC / "include").glob("*.h"))):
        h.update(str(p.relative_to(ROOT)).encode())
        h.update(b"\0")
        h.update(p.read_bytes())
    return h.hexdigest()


def build_defs() -> str:
    """The preprocessor definitions of this build mode (debug checks, dev ablations, A/B defs)."""
    return " ".join(f for f in HIP_FLAGS if f.startswith("-D"))


def stamp_text() -> str:
    return f"{source_digest()}\ndefs: {build_defs()}\n"


@contextlib.contextmanager
def _build_lock():
    """Serialise builds across processes (every data-parallel rank may trigger one): an
    exclusive flock on build/.lock; outputs are written to per-process tmp names and renamed."""
    lock = ROOT / "build" / ".lock"
    lock.parent.mkdir(parents=True, exist_ok=True)
    with open(lock, "a+") as fh:
        fcntl.flock(fh, fcntl.LOCK_EX)
        try:
            yield
        finally:
            fcntl.flock(fh, fcntl.LOCK_UN)


def build_runtime(verbose: bool = True) -> Path:
    """Host-only C++ runtime pieces (``csrc/runtime/*.cpp``: the token-shard
    loader) → ``replicann_amd/_io.so``, loaded with ctypes (no torch or HIP
    dependency, so it also works on CPU-only hosts)."""
    srcs = sorted((CSRC / "runtime").glob("*.cpp"))
    flags = ["-O3", "-std=c++17", "-fPIC", "-shared", "-pthread", "-Wall"]
    key = hashlib.sha1(("".join(s.read_text() for s in srcs) + " ".join(flags)).encode()).hexdigest()[:16]
    stamp = IO_OUT.with_suffix(".stamp")
    if IO_OUT.exists() and stamp.exists() and stamp.read_text() == key:
        return IO_OUT
    with _build_lock():
        if IO_OUT.exists() and stamp.exists() and stamp.read_text() == key:  # another process built it
            return IO_OUT
        cxx = os.environ.get("CXX") or shutil.which("g++") or "/opt/rocm/llvm/bin/clang++"
        tmp = f"{IO_OUT}.tmp.{os.getpid()}"
        r = subprocess.run([cxx, *flags, *map(str, srcs), "-o", tmp], capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"runtime build failed:\n{r.stderr[-6000:]}")
        os.replace(tmp, IO_OUT)
        stamp.write_text(key)
    if verbose:
        print(f"[replicann build] linked {IO_OUT}")
    return IO_OUT


def build(verbose: bool = True, jobs: int | None = None) -> Path:
    """Compile every kernel + binding and link ``_C.so`` (plus the host runtime
    ``_io.so``). Returns the ``_C.so`` path."""
    build_runtime(verbose)
    BUILD.mkdir(parents=True, exist_ok=True)
    with _build_lock():
        return _build_locked(verbose, jobs)


def _build_locked(verbose, jobs):
    torch_inc, torch_lib = _torch_paths()
    hdr = _headers_digest()
    # kernels (device code) + host-only bindings; csrc/comm is the native RCCL communicator
    srcs = _sources()
    jobs = jobs or min(8, os.cpu_count() or 4)
    with ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, hdr, torch_inc), srcs))
    link_key = hashlib.sha1("".join(o.name for o in objs).encode()).hexdigest()[:16]
    stamp = OUT.with_suffix(".stamp")
    digest = stamp_text()
    if OUT.exists() and stamp.exists() and stamp.read_text() == link_key:
        if not SRC_STAMP.exists() or SRC_STAMP.read_text() != digest:
            SRC_STAMP.write_text(digest)
        if verbose:
            print(f"[replicann build] up to date: {OUT}")
        return OUT
    tmp = f"{OUT}.tmp.{os.getpid()}"
    cmd = [_hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", *map(str, objs), "-o", tmp,
           f"-L{torch_lib}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip",
           f"-Wl,-rpath,{torch_lib}", f"-L{ROCM}/lib", "-lrccl", f"-Wl,-rpath,{ROCM}/lib"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stderr[-6000:]}")
    os.replace(tmp, OUT)
    stamp.write_text(link_key)
    SRC_STAMP.write_text(digest)
    if verbose:
        print(f"[replicann build] linked {OUT} from {len(objs)} objects")
    return OUT


if __name__ == "__main__":
    build()
    sys.exit(0)
