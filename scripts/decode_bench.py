"""GPT-2 KV-cache decoding throughput on one MI355X (random-init weights, bf16, greedy).

For each batch size and for the eager and the hipGraph-replayed one-token step: one untimed
generate (GEMM autotuning of the prefill / decode shapes, graph capture) and a timed generate of
``--new`` tokens; the prompt pass alone is timed once after the first warm-up.  One JSON line per (batch, step form): prefill ms, ms per
decode step (generate time minus the prefill, over the steps), generated tokens/s over the batch.

    python scripts/decode_bench.py --model gpt2-small --batches 1,16,64 --prompt 128 --new 128
"""

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="gpt2-small")
    ap.add_argument("--batches", default="1,16,64")
    ap.add_argument("--prompt", type=int, default=128)
    ap.add_argument("--new", type=int, default=128)
    a = ap.parse_args()
    from replicann_amd import _ext
    from replicann_amd.models.blocks import KVCache
    from replicann_amd.training import build_model
    from replicann_amd.tuning import load_committed
    if not _ext.available():
        raise RuntimeError(f"native extension missing: {_ext.load_error()}")
    dev = torch.device("cuda")
    load_committed(a.model)
    torch.manual_seed(0)
    m = build_model(a.model).to(dev)
    for p in m.parameters():
        p.data = p.data.to(torch.bfloat16)
    m.eval()
    for B in [int(b) for b in a.batches.split(",")]:
        idx = torch.randint(0, m.config.vocab_size, (B, a.prompt), device=dev)
        prefill = None
        for graph in (False, True):
            m.generate(idx, a.new, temperature=0, graph=graph)  # warm-up: tunes the decode GEMM shapes
            torch.cuda.synchronize()
            if prefill is None:  # the prompt pass alone, with its GEMM shapes tuned by the warm-up
                t0 = time.perf_counter()
                m.decode_step(idx, KVCache(m.config.n_layer, a.prompt + a.new))
                torch.cuda.synchronize()
                prefill = time.perf_counter() - t0
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            out = m.generate(idx, a.new, temperature=0, graph=graph)
            torch.cuda.synchronize()
            total = time.perf_counter() - t0
            step_ms = (total - prefill) / max(1, a.new - 1) * 1e3
            print(json.dumps({"model": a.model, "batch": B, "prompt": a.prompt, "new_tokens": a.new,
                              "decode_step": "hipGraph replay" if graph else "eager",
                              "prefill_ms": round(prefill * 1e3, 3), "decode_ms_per_step": round(step_ms, 3),
                              "generated_tokens_per_s": round(B * a.new / total, 1),
                              "out_shape": list(out.shape), "dtype": "bf16", "weights": "random init"}), flush=True)

if __name__ == "__main__":
    main()
