"""The native RCCL communicator (csrc/comm/rccl_comm.cpp) and the data-parallel step on RCCL,
rehearsed on ONE MI355X (RCCL refuses two ranks on one device, so these run a one-rank
communicator / process group; the multi-rank reducer logic is covered over gloo in
test_ddp.py / test_ddp_gpu.py).

* every collective of NativeComm on a one-rank communicator (identity / copy semantics),
  its stream fork/join ordering, and a collective captured into a hipGraph and replayed;
* the full GPT-2 DDP step (``ddp="on"``: bucket hooks, fp32 widening, tied-weight split,
  collectives, optimizer reading the reduction buffer) over (a) the native communicator
  and (b) torch.distributed's ProcessGroupNCCL: both give bitwise the same trajectory, it
  stays within bf16 rounding of the non-DDP step, and the native one also runs as ONE
  captured hipGraph."""

import os
import socket

import pytest
import torch
import torch.distributed as dist

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture
def one_rank_pg(monkeypatch):
    """A one-process nccl (= RCCL) group, destroyed afterwards."""
    monkeypatch.setenv("MASTER_ADDR", "127.0.0.1")
    monkeypatch.setenv("MASTER_PORT", str(_free_port()))
    monkeypatch.setenv("RANK", "0")
    monkeypatch.setenv("WORLD_SIZE", "1")
    monkeypatch.setenv("LOCAL_RANK", "0")
    yield
    if dist.is_initialized():
        dist.destroy_process_group()


def test_native_comm_collectives_one_rank():
    from replicann_amd.parallel.comm import NativeComm

    c = NativeComm(device="cuda:0")
    try:
        x = torch.randn(1 << 20, device="cuda")
        ref = x.clone()
        c.all_reduce(x)
        c.wait()
        assert torch.equal(x, ref)
        c.all_reduce(x, op="max")
        b = torch.randn(4096, device="cuda", dtype=torch.bfloat16)
        bref = b.clone()
        c.broadcast(b, 0)
        out = torch.empty_like(b)
        c.all_gather(b, out)
        rs = torch.empty_like(b)
        c.reduce_scatter(b, rs)
        c.wait()
        torch.cuda.synchronize()
        assert torch.equal(b, bref) and torch.equal(out, bref) and torch.equal(rs, bref)
        info = c.info()
        assert info["collectives"] == 5 and info["world"] == 1 and not info["failed"]
        c.synchronize()
    finally:
        c.close()


def test_native_comm_stream_ordering():
    """The collective runs after the compute stream's producer and before its consumer."""
    from replicann_amd.parallel.comm import NativeComm

    c = NativeComm(device="cuda:0")
    try:
        a = torch.randn(8 << 20, device="cuda")
        for _ in range(3):
            y = a * 2.0          # producer on the compute stream
            c.all_reduce(y)      # comm stream forks after it
            c.wait()             # compute stream joins
            z = y + 1.0          # consumer
        torch.cuda.synchronize()
        assert torch.equal(z, a * 2.0 + 1.0)
    finally:
        c.close()


def test_native_comm_graph_capture():
    from replicann_amd.parallel.comm import NativeComm

    c = NativeComm(device="cuda:0")
    try:
        x = torch.zeros(1 << 16, device="cuda")
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):  # warm-up outside the capture
            y = x + 1.0
            c.all_reduce(y)
            c.wait()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            y = x + 1.0
            c.all_reduce(y)
            c.wait()
            z = y * 3.0
        for v in (1.0, 5.0):
            x.fill_(v)
            g.replay()
            torch.cuda.synchronize()
            assert torch.equal(z, torch.full_like(x, (v + 1.0) * 3.0))
    finally:
        c.close()


def _run(cfg_kw, steps=4, skip_tune=False):
    from replicann_amd.training import TrainConfig, Trainer

    if cfg_kw.get("graph") != "off":
        # a capture may follow ProcessGroupNCCL collectives of an earlier run: let that group's watchdog
        # thread retire their (completed) works first — its event queries fail during a global capture
        import time
        torch.cuda.synchronize()
        time.sleep(0.5)

    cfg = TrainConfig(model="gpt2-tiny", batch_size=4, seq_len=128, steps=100, warmup_steps=1, lr=1e-3,
                      log_every=10**9, bucket_mb=0.5, seed=3, **cfg_kw)
    tr = Trainer(cfg)
    tr._tuned = tr._tuned or skip_tune
    losses = [float(tr.step()) for _ in range(steps)]
    torch.cuda.synchronize()
    out = (losses, tr.flat.data.float().clone(), tr._graph is not None,
           tr.ddp.comm.name if tr.ddp is not None else None,
           tr.ddp.launched_in_backward if tr.ddp is not None else 0)
    if tr.ddp is not None:
        tr.ddp.comm.close()
    return out


def test_ddp_step_native_vs_torch_rccl(one_rank_pg):
    base_l, base_w, _, _, _ = _run(dict(graph="off"))
    nat_l, nat_w, nat_g, nat_c, nat_hooked = _run(dict(graph="off", ddp="on", comm="native"))
    assert dist.is_initialized() and dist.get_backend() == "nccl"
    tor_l, tor_w, _, tor_c, _ = _run(dict(graph="off", ddp="on", comm="torch"))
    assert (nat_c, tor_c, nat_g) == ("native", "torch", False)
    assert nat_hooked > 0  # buckets were issued from gradient hooks during the backward
    assert nat_l == tor_l and torch.equal(nat_w, tor_w)  # same reduction, two transports
    # vs the non-DDP step: the tied wte's two contributions are summed in fp32 instead of bf16
    for a, b in zip(nat_l, base_l):
        assert abs(a - b) <= 2e-2 * abs(b), (nat_l, base_l)
    assert (nat_w - base_w).abs().max().item() < 5e-2


def test_ddp_step_native_graph_matches_eager(one_rank_pg):
    eag_l, eag_w, eag_g, _, _ = _run(dict(graph="off", ddp="on", comm="native"))
    gr_l, gr_w, gr_g, gr_c, _ = _run(dict(graph="auto", ddp="on", comm="native"))
    assert gr_c == "native" and gr_g and not eag_g  # the whole DDP step replays as one hipGraph
    assert eag_l == gr_l and torch.equal(eag_w, gr_w)


def test_ddp_pre_step_tuning_pass_is_invisible(one_rank_pg):
    """The reducer-suspended autotuning pass before the first DDP step changes nothing the
    training sees (batch stream, gradients, optimizer state, RNG)."""
    a_l, a_w, _, _, _ = _run(dict(graph="off", ddp="on", comm="native"))
    b_l, b_w, _, _, _ = _run(dict(graph="off", ddp="on", comm="native"), skip_tune=True)
    assert a_l == b_l and torch.equal(a_w, b_w)


def test_proxy_comm_keeps_data_and_orders_streams():
    """REPLICANN_COMM=proxy: the collectives move the emulated ring volume through HBM on the comm
    stream (values unchanged at world 1), stream-ordered like the real ones, and capturable."""
    from replicann_amd.parallel.comm import NativeComm

    c = NativeComm(device="cuda:0", proxy=True)
    try:
        assert c.name == "proxy" and c.proxy_world >= 2
        a = torch.randn(4 << 20, device="cuda")
        for _ in range(3):
            y = a * 2.0
            c.all_reduce(y)
            c.wait()
            z = y + 1.0
        b = torch.randn(4096, device="cuda", dtype=torch.bfloat16)
        out = torch.empty_like(b)
        c.all_gather(b, out)
        c.broadcast(b, 0)
        c.wait()
        torch.cuda.synchronize()
        assert torch.equal(z, a * 2.0 + 1.0) and torch.equal(out, b)
        assert c.info()["collectives"] == 5
    finally:
        c.close()


def test_ddp_step_proxy_matches_native_and_enables_queue(one_rank_pg, monkeypatch):
    torch.ops.replicann.gemm_set_sched(0)
    monkeypatch.setenv("REPLICANN_GEMM_SCHED", "dynamic")  # opt-in (static is the measured default)
    nat_l, nat_w, _, _, _ = _run(dict(graph="off", ddp="on", comm="native"))
    assert torch.ops.replicann.gemm_get_sched() == 0  # a one-rank real group runs no collective beside GEMMs
    px_l, px_w, px_g, px_c, _ = _run(dict(graph="auto", ddp="on", comm="proxy"))
    try:
        assert px_c == "proxy" and px_g  # capturable like the native communicator
        assert torch.ops.replicann.gemm_get_sched() == 1  # dynamic tile queue while collectives overlap (opt-in)
        assert px_l == nat_l and torch.equal(px_w, nat_w)  # (the queue changes no output bit)
    finally:
        torch.ops.replicann.gemm_set_sched(0)
        torch.ops.replicann.gemm_set_reserve(0)


def test_ddp_step_rsag_native_torch_graph(one_rank_pg):
    """reduce_dtype="rsag" (fp32 reduce-scatter -> bf16 narrow -> bf16 all-gather per bucket): the
    native communicator (narrow on its comm stream) and ProcessGroupNCCL (narrow on a side stream)
    give the same bits, the native step captures into one hipGraph with the same result, and the
    training tracks the fp32 all-reduce step (one bf16 rounding of the summed gradient)."""
    fp_l, fp_w, _, _, _ = _run(dict(graph="off", ddp="on", comm="native", reduce_dtype="fp32"))
    nat_l, nat_w, _, nat_c, hooked = _run(dict(graph="off", ddp="on", comm="native", reduce_dtype="rsag"))
    # (captured before any ProcessGroupNCCL run: that group's watchdog thread queries its works' events
    # and a global-mode capture in progress makes those queries fail)
    gr_l, gr_w, gr_g, _, _ = _run(dict(graph="auto", ddp="on", comm="native", reduce_dtype="rsag"))
    tor_l, tor_w, _, tor_c, _ = _run(dict(graph="off", ddp="on", comm="torch", reduce_dtype="rsag"))
    assert (nat_c, tor_c) == ("native", "torch") and hooked > 0 and gr_g
    assert nat_l == tor_l and torch.equal(nat_w, tor_w)
    assert nat_l == gr_l and torch.equal(nat_w, gr_w)
    for a, b in zip(nat_l, fp_l):
        assert abs(a - b) <= 2e-2 * abs(b), (nat_l, fp_l)
    assert (nat_w - fp_w).abs().max().item() < 5e-2


def test_proxy_reduce_scatter_narrow_all_gather():
    """Proxy communicator: reduce-scatter (world 1: a copy) then narrow + bf16 all-gather returns the
    bf16-rounded input, stream-ordered on the comm stream."""
    from replicann_amd.parallel.comm import NativeComm

    c = NativeComm(device="cuda:0", proxy=True)
    try:
        a = torch.randn(1 << 20, device="cuda")
        s32 = torch.empty_like(a)
        s16 = torch.empty(a.numel(), device="cuda", dtype=torch.bfloat16)
        full = torch.empty_like(s16)
        c.reduce_scatter(a, s32)
        c.narrow_all_gather(s32, s16, full)
        c.wait()
        torch.cuda.synchronize()
        assert torch.equal(full, a.to(torch.bfloat16)) and torch.equal(s16, full)
    finally:
        c.close()


def test_ddp_window_schedule_matches_eager(one_rank_pg):
    """schedule="window" (collectives queued until the next attention backward, at most window_mb per
    window, the rest in finish()) and "end" change WHEN the reductions run, not their result: losses and
    weights equal the eager schedule's, for the fp32 all-reduce and rsag, native and torch transports."""
    refs = {}
    for red in ("fp32", "rsag"):  # every capture first (see the rsag test), then the torch transport
        ref_l, ref_w, _, _, _ = _run(dict(graph="off", ddp="on", comm="native", reduce_dtype=red))
        refs[red] = (ref_l, ref_w)
        gl, gw, gg, _, _ = _run(dict(graph="auto", ddp="on", comm="native", reduce_dtype=red, ddp_schedule="window"))
        assert gg and gl == ref_l and torch.equal(gw, ref_w)  # window schedule captures into one hipGraph
    for red in ("fp32", "rsag"):
        ref_l, ref_w = refs[red]
        for comm in ("native", "torch"):
            for sched in ("window", "end"):
                l, w, _, _, _ = _run(dict(graph="off", ddp="on", comm=comm, reduce_dtype=red, ddp_schedule=sched))
                assert l == ref_l and torch.equal(w, ref_w), (red, comm, sched)
