"""N24 benchmark harness contract (CPU/gloo path): ``bench.py --gpus N`` launches its own N
ranks when no external launcher did, reports the communicator's world size, and refuses to
report a number when the ranks it got do not match ``--gpus``."""

import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*args, env=None):
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    e.update(env or {})
    e["PYTHONPATH"] = ROOT
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], cwd="/tmp", env=e,
                          capture_output=True, text=True, timeout=600)


def test_bench_spawns_its_own_ranks():
    r = _bench("--gpus", "2", "--model", "mlp", "--device", "cpu", "--steps", "2", "--warmup", "1")
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["comm_world"] == 2
    assert out["config"]["parallelism"] == "dp2" and out["config"]["global_batch"] == 2 * out["config"]["micro_batch_per_gpu"]
    assert out["config"]["hipgraph"] == [False, False]
    assert out["steps"] == 2 and out["warmup"] == 1 and out["value"] > 0


def test_bench_rank_mismatch_fails():
    r = _bench("--gpus", "2", "--model", "mlp", "--device", "cpu", "--steps", "1", "--warmup", "0",
               env={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


def test_bench_gpt2_eight_ranks_self_diagnosing():
    """The headline model family's data-parallel path (GPT-2 with its tied wte: the LM-head and
    embedding contributions reduced separately) through the real harness at 8 ranks on gloo: one JSON
    line with comm_world == 8 and the record a first multi-GPU run needs (exposed comm, collectives /
    bytes, the schedule auto resolved to, rank spread).  (On the CPU the gradients are fp32, so the
    reducer runs its in-place all-reduce; rsag and the attention-backward windows are the bf16 GPU
    path, rehearsed on one card by tests/test_ddp_gpu.py.)"""
    r = _bench("--gpus", "8", "--model", "gpt2-tiny", "--device", "cpu", "--steps", "1", "--warmup", "1",
               "--seq", "64", "--batch", "2", env={"OMP_NUM_THREADS": "1"})
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    c = out["config"]
    assert out["n_gpus"] == 8 and c["comm_world"] == 8 and c["parallelism"] == "dp8"
    d = c["ddp_diag"]
    assert d["collectives_per_step"] > 0 and d["comm_gbytes_per_step"] > 0
    assert d["allreduce_wait_ms_max"] is not None and d["allreduce_wait_ms_max"] >= d["allreduce_wait_ms_min"]
    assert d["schedule"].startswith("auto->") and d["reduce"]
    assert len(d["rank_ms_per_step"]) == 8 and d["rank_ms_spread"] >= 0
    assert "backward_ms" in d["step_phases_ms_rank0"]
