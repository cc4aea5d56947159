"""Native token-shard loader (csrc/runtime/token_loader.cpp via utils/token_data.py), CPU tier.

Checks window contents against the shard bytes (random and eval modes,
uint16 / uint32, multiple shards), determinism independent of thread count,
resume at a batch index, rank-disjoint eval windows, argument errors, and a
GPT-2 training run fed from a shard through the trainer's ``data=`` option."""

import numpy as np
import pytest
import torch

from replicann_amd.utils.token_data import TokenFileLM, write_token_shard


def _is_window(row, shards):
    for s in shards:
        n = len(row)
        # candidate starts where the first token matches
        for st in np.nonzero(s[: len(s) - n + 1] == row[0])[0]:
            if np.array_equal(s[st:st + n], row):
                return True
    return False


@pytest.fixture
def shards(tmp_path):
    rng = np.random.default_rng(0)
    a = rng.integers(0, 50000, 5000)
    b = rng.integers(0, 50000, 777)
    pa = write_token_shard(tmp_path / "a.bin", a)
    pb = write_token_shard(tmp_path / "b.bin", b)
    return [pa, pb], [a, b]


def test_train_windows_are_shard_slices(shards):
    paths, data = shards
    ld = TokenFileLM(paths, 4, 32, "cpu", seed=3)
    assert ld.num_tokens == 5777
    for _ in range(5):
        x, y = next(ld)
        assert x.shape == (4, 32) and y.shape == (4, 32) and x.dtype == torch.int64
        torch.testing.assert_close(x[:, 1:], y[:, :-1])
        full = torch.cat([x, y[:, -1:]], 1).numpy()
        for row in full:
            assert _is_window(row, data)


def test_deterministic_across_threads_and_resume(shards):
    paths, _ = shards
    a = TokenFileLM(paths, 3, 16, "cpu", seed=11, threads=1, prefetch=2)
    b = TokenFileLM(paths, 3, 16, "cpu", seed=11, threads=4, prefetch=8)
    seq_a = [next(a)[0] for _ in range(12)]
    seq_b = [next(b)[0] for _ in range(12)]
    for u, v in zip(seq_a, seq_b):
        assert torch.equal(u, v)
    r = TokenFileLM(paths, 3, 16, "cpu", seed=11, start_batch=7)
    for k in range(7, 12):
        assert torch.equal(next(r)[0], seq_a[k])
    assert r.batch_index == 12
    c = TokenFileLM(paths, 3, 16, "cpu", seed=12)
    assert not torch.equal(next(c)[0], seq_a[0])
    d = TokenFileLM(paths, 3, 16, "cpu", seed=11, rank=1, world=2)
    assert not torch.equal(next(d)[0], seq_a[0])


def test_eval_windows_cover_shards_round_robin(tmp_path):
    tok = np.arange(1, 4 * 10 + 2, dtype=np.int64)   # 41 tokens, T=10 → 4 windows
    p = write_token_shard(tmp_path / "s.bin", tok, dtype=np.uint32)
    r0 = TokenFileLM(p, 1, 10, "cpu", mode="eval", dtype="uint32", rank=0, world=2)
    r1 = TokenFileLM(p, 1, 10, "cpu", mode="eval", dtype="uint32", rank=1, world=2)
    assert r0.num_windows == 4
    seen = []
    for _ in range(2):
        for ld in (r0, r1):
            x, y = next(ld)
            seen.append(int(x[0, 0]))
            assert torch.equal(y[0], x[0] + 1)
    assert seen == [1, 11, 21, 31]
    x, _ = next(r0)               # wraps to window 0 of the next epoch
    assert int(x[0, 0]) == 1


def test_errors(tmp_path):
    p = write_token_shard(tmp_path / "tiny.bin", np.arange(5))
    with pytest.raises(ValueError, match="shorter"):
        TokenFileLM(p, 2, 8, "cpu")
    with pytest.raises(ValueError, match="cannot open"):
        TokenFileLM(tmp_path / "missing.bin", 2, 2, "cpu")
    with pytest.raises(ValueError):
        write_token_shard(tmp_path / "neg.bin", np.array([-1, 2]))
    big = write_token_shard(tmp_path / "big.bin", np.full(64, 1000))
    ld = TokenFileLM(big, 2, 8, "cpu", vocab=512)
    with pytest.raises(ValueError, match="vocab"):
        next(ld)


def test_trainer_reads_token_shards(tmp_path):
    from replicann_amd.training import TrainConfig, Trainer
    rng = np.random.default_rng(1)
    # a learnable stream: a fixed cycle of 64 token ids
    cyc = rng.integers(0, 256, 64)
    write_token_shard(tmp_path / "train_000.bin", np.tile(cyc, 200))
    cfg = TrainConfig(model="gpt2-tiny", device="cpu", dtype="fp32", batch_size=4, seq_len=32, steps=12,
                      warmup_steps=2, lr=3e-3, log_every=10**9, graph="off", data=str(tmp_path / "train_*.bin"),
                      model_kwargs=dict(n_embd=64, vocab_size=256, vocab_pad=256, block_size=32))
    tr = Trainer(cfg)
    assert isinstance(tr.data, TokenFileLM)
    losses = [float(tr.step()) for _ in range(12)]
    assert losses[-1] < losses[0] - 0.5, losses


@pytest.mark.gpu
def test_pinned_h2d_stream_matches_cpu(shards):
    """cuda path: pinned ring + non-blocking copies deliver the same batches as the CPU path."""
    paths, _ = shards
    g = TokenFileLM(paths, 8, 64, "cuda", seed=5, pinned=2)
    c = TokenFileLM(paths, 8, 64, "cpu", seed=5)
    outs = [next(g) for _ in range(6)]       # more batches than pinned buffers: exercises buffer reuse
    torch.cuda.synchronize()
    for x, y in outs:
        cx, cy = next(c)
        assert x.is_cuda and torch.equal(x.cpu(), cx) and torch.equal(y.cpu(), cy)


@pytest.mark.parametrize("san", ["thread", "address,undefined"])
def test_loader_under_sanitizers(tmp_path, san):
    """Host sanitizers over the native loader (8 workers, 3-slot ring, destroy with parked workers)."""
    import shutil
    import subprocess
    from pathlib import Path
    if shutil.which("g++") is None:
        pytest.skip("g++ not available")
    rt = Path(__file__).resolve().parent.parent / "csrc" / "runtime"
    exe = tmp_path / "stress"
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", f"-fsanitize={san}", "-pthread", str(rt / "token_loader.cpp"),
                    str(rt / "tests" / "loader_stress.cpp"), "-o", str(exe)], check=True, timeout=120)
    shard = write_token_shard(tmp_path / "s.bin", np.random.default_rng(0).integers(0, 65536, 100000))
    r = subprocess.run([str(exe), str(shard)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "loader stress ok" in r.stdout, r.stderr[-3000:]
