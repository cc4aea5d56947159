"""All-reduce bandwidth of the two collective back-ends over RCCL (xGMI on one node):

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 scripts/comm_bench.py

For each message size (fp32, the DDP reduction dtype) and back-end (native communicator,
torch ProcessGroupNCCL) it times `iters` back-to-back all-reduces between barriers and prints, on
rank 0, one JSON line: time, algorithm bandwidth (bytes / t) and bus bandwidth
(2 (n-1)/n · bytes / t, the per-link figure a ring achieves).  The DDP bucket size
(TrainConfig.bucket_mb, default 64 MB) should sit where busbw has flattened; RCCL's own knobs
(NCCL_MIN_NCHANNELS / NCCL_MAX_NCHANNELS, NCCL_ALGO) can be A/B'd with the same command.
Runs at world 1 too (a one-rank communicator: a local copy — a smoke test, not a bandwidth)."""

import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from replicann_amd.parallel import init_distributed  # noqa: E402
from replicann_amd.parallel.comm import NativeComm, TorchComm  # noqa: E402


def main():
    rank, local, world, dev = init_distributed(force=True)
    sizes_mb = [float(s) for s in (sys.argv[1].split(",") if len(sys.argv) > 1 else "1,4,16,64,256".split(","))]
    iters = int(os.environ.get("COMM_BENCH_ITERS", "20"))
    comms = {"native": NativeComm(device=dev), "torch": TorchComm()}
    for mb in sizes_mb:
        n = int(mb * 1024 * 1024 / 4)
        x = torch.ones(n, device=dev)
        for name, c in comms.items():
            for _ in range(3):
                c.all_reduce(x)
            c.wait()
            torch.cuda.synchronize(dev)
            dist.barrier()
            t0 = time.perf_counter()
            for _ in range(iters):
                c.all_reduce(x)
            c.wait()
            torch.cuda.synchronize(dev)
            dt = (time.perf_counter() - t0) / iters
            t = torch.tensor([dt], device=dev, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dt = float(t)
            b = n * 4
            if rank == 0:
                print(json.dumps({"comm": name, "world": world, "MB": mb, "ms": round(dt * 1e3, 4),
                                  "algbw_GBps": round(b / dt / 1e9, 1),
                                  "busbw_GBps": round(2 * (world - 1) / world * b / dt / 1e9, 1)}), flush=True)
    comms["native"].close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
