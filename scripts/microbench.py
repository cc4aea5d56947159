"""Per-op microbenchmarks on the GPT-2-small training shapes (B=16, T=1024):
our HIP kernels vs the stock PyTorch-ROCm path (hipBLASLt GEMM, ATen SDPA,
ATen LayerNorm / cross-entropy), interleaved in one process (§5.4 rule 24),
random data.  Prints one JSON line per op; writes gpurun_out/microbench.json."""

import json
import math
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from replicann_amd import ops  # noqa: E402


def timeit(fn, iters=20, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(iters):
        fn()
    ev[1].record()
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]) / iters


def bf(*s):
    return torch.randn(*s, device="cuda", dtype=torch.bfloat16)


def main():
    torch.manual_seed(0)
    M = 16 * 1024
    res = []
    want = set(sys.argv[1:]) or {"gemm", "fp8", "attn", "ln", "xent"}
    gemms = [  # name, M, N, K, layout
        ("qkv_fwd", M, 2304, 768, "nt"), ("proj_fwd", M, 768, 768, "nt"), ("fc_fwd", M, 3072, 768, "nt"),
        ("fc2_fwd", M, 768, 3072, "nt"), ("lmhead_fwd", M, 50304, 768, "nt"),
        ("fc_dgrad", M, 768, 3072, "nn"), ("qkv_dgrad", M, 768, 2304, "nn"), ("lmhead_dgrad", M, 768, 50304, "nn"),
        ("fc_wgrad", 3072, 768, M, "tn"), ("qkv_wgrad", 2304, 768, M, "tn"), ("proj_wgrad", 768, 768, M, "tn"),
        ("lmhead_wgrad", 50304, 768, M, "tn"),
    ]
    for name, m, n, k, lay in (gemms if "gemm" in want else []):
        ta, tb = lay[0] == "t", lay[1] == "t"
        a = bf(k, m) if ta else bf(m, k)
        b = bf(n, k) if tb else bf(k, n)
        A = a.t() if ta else a
        B = b.t() if tb else b
        from replicann_amd.ops.linear import _pick_split_k
        sk = _pick_split_k(m, n, k) if ta else 0
        ref = lambda: A @ B
        fl = 2 * m * n * k
        t_r = min(timeit(ref) for _ in range(3))
        cfg_t = {}
        for cfg in (-1, 0, 1, 2, 5, 6, 8) + (() if ta else (7,)):
            for s_ in (sorted({-1, 1, 2, 4}) if ta else [0]) if cfg != 7 else [0]:
                ours = lambda: ops.gemm(a, b, ta=ta, tb=tb, split_k=s_, cfg=cfg)
                err = ((ours().float() - ref().float()).norm() / ref().float().norm()).item()
                cfg_t[f"c{cfg}s{s_}"] = (min(timeit(ours) for _ in range(2)), err)
        auto = cfg_t["c-1s-1"] if ta else cfg_t["c-1s0"]
        best = min(cfg_t.items(), key=lambda kv: kv[1][0])
        r = dict(op=f"gemm_{name}", M=m, N=n, K=k, layout=lay, split_k=sk, ours_ms=auto[0], torch_ms=t_r,
                 ours_tflops=fl / auto[0] / 1e9, torch_tflops=fl / t_r / 1e9, rel_err=auto[1],
                 best=best[0], best_tflops=fl / best[1][0] / 1e9,
                 all_tflops={kk: round(fl / v[0] / 1e9) for kk, v in cfg_t.items()})
        print(json.dumps(r), flush=True)
        res.append(r)
    # fp8 (block-scaled MFMA) vs bf16 on GPT-2-medium forward shapes
    for name, m, n, k in ((("med_qkv", M, 3072, 1024), ("med_fc", M, 4096, 1024), ("med_fc2", M, 1024, 4096),
                           ("med_proj", M, 1024, 1024)) if "fp8" in want else ()):
        a, b = bf(m, k), bf(n, k)
        qa, sa = ops.quantize_fp8(a)
        qb, sb = ops.quantize_fp8(b)
        f8 = lambda: torch.ops.replicann.gemm_fp8(qa, qb, sa, sb, None, None, 0, None)
        q8 = lambda: ops.quantize_fp8(a)
        b16 = lambda: ops.gemm(a, b, tb=True)
        fl = 2 * m * n * k
        t8, tq, t16 = (min(timeit(f) for _ in range(2)) for f in (f8, q8, b16))
        r = dict(op=f"fp8_{name}", fp8_gemm_tflops=fl / t8 / 1e9, bf16_gemm_tflops=fl / t16 / 1e9,
                 fp8_ms=t8, quant_act_ms=tq, bf16_ms=t16)
        print(json.dumps(r), flush=True)
        res.append(r)
    # attention fwd / bwd (B=16, H=12, T=1024, D=64, causal)
    B, T, H, D = 16, 1024, 12, 64
    attn_cases = ("attn_fwd", "attn_bwd") if "attn" in want else ()
    qkv = bf(B, T, 3, H, D).requires_grad_()
    q, k, v = [t.detach().transpose(1, 2).contiguous().requires_grad_() for t in qkv.unbind(2)]
    go = bf(B, T, H, D)
    f_o = lambda: ops.attention_packed(qkv, causal=True)
    f_r = lambda: F.scaled_dot_product_attention(q, k, v, is_causal=True)
    out_o = f_o()
    out_r = f_r()
    b_o = lambda: torch.autograd.grad(out_o, qkv, go, retain_graph=True)
    gr = go.transpose(1, 2).contiguous()
    b_r = lambda: torch.autograd.grad(out_r, (q, k, v), gr, retain_graph=True)
    fl_f = 4 * B * H * T * T * D / 2
    for nm, fo, fr, fl in [c for c in (("attn_fwd", f_o, f_r, fl_f), ("attn_bwd", b_o, b_r, 2.5 * fl_f))
                           if c[0] in attn_cases]:
        t_o = min(timeit(fo) for _ in range(3))
        t_r = min(timeit(fr) for _ in range(3))
        r = dict(op=nm, ours_ms=t_o, torch_ms=t_r, ours_tflops=fl / t_o / 1e9, torch_tflops=fl / t_r / 1e9)
        print(json.dumps(r), flush=True)
        res.append(r)
    # LayerNorm, cross-entropy
    if "ln" not in want and "xent" not in want:
        return _dump(res)
    x, w, bb = bf(M, 768), bf(768), bf(768)
    t_o = min(timeit(lambda: ops.layer_norm(x, w, bb)) for _ in range(3))
    t_r = min(timeit(lambda: F.layer_norm(x, (768,), w, bb)) for _ in range(3))
    r = dict(op="layernorm_fwd", ours_ms=t_o, torch_ms=t_r, gbps=2 * x.numel() * 2 / t_o / 1e6)
    print(json.dumps(r), flush=True)
    res.append(r)
    logits = bf(M, 50304)
    tgt = torch.randint(0, 50257, (M,), device="cuda")
    t_o = min(timeit(lambda: ops.cross_entropy(logits, tgt, n_valid_cols=50257)) for _ in range(3))
    t_r = min(timeit(lambda: F.cross_entropy(logits[:, :50257].float(), tgt)) for _ in range(3))
    r = dict(op="xent_fwd", ours_ms=t_o, torch_ms=t_r, gbps=logits.numel() * 2 / t_o / 1e6)
    print(json.dumps(r), flush=True)
    res.append(r)
    _dump(res)


def _dump(res):
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/microbench.json", "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
