"""Communicator layer: LocalComm, ThreadComm, TorchDistComm (gloo), backend resolution,
rank-divergence detection, the compat shim's comm functions."""
import os

import pytest
import torch

from _dist import run_gloo
from xdot.utils import comm as C


def test_resolve_backend():
    assert C.resolve_backend("rccl") == "nccl"
    assert C.resolve_backend("nccl") == "nccl"
    assert C.resolve_backend("gloo") == "gloo"
    assert C.resolve_backend("auto") in ("nccl", "gloo")
    with pytest.raises(ValueError):
        C.resolve_backend("mpi")


def test_local_comm_semantics():
    c = C.LocalComm()
    x = torch.arange(6.0)
    out = torch.empty(6)
    c.all_gather_into(out, x)
    assert torch.equal(out, x)
    h = c.reduce_scatter(out, x * 2, async_op=True)
    assert torch.equal(h.wait(), x * 2)
    assert c.all_gather_object({"a": 1}) == [{"a": 1}]
    c.barrier()


def test_default_is_single_rank_without_env(monkeypatch):
    for k in ("WORLD_SIZE", "MASTER_ADDR", "RANK"):
        monkeypatch.delenv(k, raising=False)
    with C.use_comm(C.LocalComm()):
        assert C.get_world_size() == 1 and C.get_rank() == 0 and C.is_main_process()
        C.synchronize()


@pytest.mark.parametrize("ws", [2, 3])
def test_thread_comm_collectives(ws):
    def body(r):
        c = C.get_comm()
        assert c.rank == r and c.world_size == ws
        x = torch.full((2, 3), float(r))
        out = torch.empty(ws, 2, 3)
        c.all_gather_into(out, x)
        assert all(torch.all(out[j] == j) for j in range(ws))
        send = torch.arange(ws * 4, dtype=torch.float32) * (r + 1)
        rs = torch.empty(4)
        c.reduce_scatter(rs, send)
        tot = sum(range(1, ws + 1))
        assert torch.equal(rs, torch.arange(r * 4, r * 4 + 4, dtype=torch.float32) * tot)
        t = torch.tensor([float(r)])
        c.all_reduce(t, "max")
        assert t.item() == ws - 1
        a = torch.tensor([float(r)])
        c.all_reduce(a, "avg")
        assert a.item() == sum(range(ws)) / ws
        b = torch.tensor([float(r + 10)])
        c.broadcast(b, src=1)
        assert b.item() == 11.0
        assert c.all_gather_object(r * 2) == [2 * j for j in range(ws)]
        got = torch.empty(3)
        c.sendrecv(torch.full((3,), float(r)), got, (r + 1) % ws, (r - 1) % ws)  # one ring hop
        assert torch.all(got == (r - 1) % ws)
        return r

    assert C.ThreadGroup(ws).run(body) == list(range(ws))


def test_thread_group_propagates_errors():
    def body(r):
        if r == 1:
            raise KeyError("boom")
        C.get_comm().barrier()

    with pytest.raises(KeyError):
        C.ThreadGroup(2, timeout=10).run(body)


def _gloo_collectives(rank, ws):
    c = C.get_comm()
    assert isinstance(c, C.TorchDistComm) and c.backend == "gloo"
    for dt in (torch.float32, torch.bfloat16, torch.int64):
        x = torch.full((5,), rank + 1).to(dt)
        out = torch.empty(ws * 5, dtype=dt)
        c.all_gather_into(out, x, async_op=True).wait()
        assert out.view(ws, 5)[:, 0].tolist() == [j + 1 for j in range(ws)]
        rs = torch.empty(5, dtype=dt)
        c.reduce_scatter(rs, torch.ones(ws * 5, dtype=dt))
        assert torch.all(rs.float() == ws)
        got = torch.empty(5, dtype=dt)  # one ring hop (isend/irecv pair)
        c.sendrecv(torch.full((5,), rank + 1).to(dt), got, (rank + 1) % ws, (rank - 1) % ws, async_op=True).wait()
        assert torch.all(got.float() == (rank - 1) % ws + 1)
    # the shim's comm functions resolve to the same communicator
    from distributed_dot_product.utils.comm import get_rank, get_world_size, is_main_process, synchronize

    assert get_rank() == rank and get_world_size() == ws and is_main_process() == (rank == 0)
    synchronize()


def test_gloo_collectives():
    run_gloo(_gloo_collectives, 2)


def test_divergence_check_threads(monkeypatch):
    from xdot.utils import checks
    from xdot.utils.env import FLAGS

    def body(r):
        x = torch.zeros(2, 3 if r == 0 else 4)
        checks.check_consistent(C.get_comm(), "op", x, force=True)

    with pytest.raises(checks.RankDivergenceError):
        C.ThreadGroup(2).run(body)

    def same(r):
        checks.check_consistent(C.get_comm(), "op", torch.zeros(2, 3), force=True)

    C.ThreadGroup(2).run(same)
    assert not FLAGS.check  # default off


def test_env_flags(monkeypatch):
    from xdot.utils.env import FLAGS

    monkeypatch.setenv("DISTRIBUTED_DOT_DEBUG", "1")
    monkeypatch.setenv("XDOT_BACKEND", "torch")
    FLAGS.reload()
    try:
        assert FLAGS.debug and FLAGS.backend == "torch"
    finally:
        monkeypatch.delenv("DISTRIBUTED_DOT_DEBUG")
        monkeypatch.delenv("XDOT_BACKEND")
        FLAGS.reload()
    assert not FLAGS.debug


def test_measure_debug_output(capsys, monkeypatch):
    from xdot.utils.env import FLAGS
    import xdot.parallel.functional as F

    monkeypatch.setenv("XDOT_DEBUG", "1")
    FLAGS.reload()
    try:
        F.distributed_matmul_nt(torch.randn(1, 4, 3), torch.randn(1, 4, 3))
    finally:
        monkeypatch.delenv("XDOT_DEBUG")
        FLAGS.reload()
    assert "distributed_matmul_nt" in capsys.readouterr().out


def test_fp32_buffer_mode_flags(monkeypatch):
    """XDOT_FP32_DS_ONLY picks which fp32 families keep only a dS buffer (flash.ds_only_wanted):
    the split family by default, both or none on request, never the wide heads."""
    from xdot.ops import flash
    from xdot.utils.env import FLAGS

    old = FLAGS.fp32_ds_only
    try:
        for mode, exact, split in (("split", False, True), ("all", True, True), ("none", False, False)):
            monkeypatch.setenv("XDOT_FP32_DS_ONLY", mode)
            FLAGS.reload()
            assert FLAGS.fp32_ds_only == mode
            assert flash.ds_only_wanted(0, 96) is exact and flash.ds_only_wanted(1, 96) is split
            assert flash.ds_only_wanted(1, 128) is split
            assert not flash.ds_only_wanted(0, 256) and not flash.ds_only_wanted(1, 384)
        monkeypatch.delenv("XDOT_FP32_DS_ONLY")
        FLAGS.reload()
        assert FLAGS.fp32_ds_only == "split"
    finally:
        FLAGS.fp32_ds_only = old
