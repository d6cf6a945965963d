"""Chunk planning and the double-buffered gather pipeline."""
import pytest
import torch

from xdot.parallel.schedule import auto_offset, gather_pipeline, plan_chunks, resolve_offset
from xdot.utils.comm import LocalComm, ThreadGroup


def test_plan_chunks():
    assert plan_chunks(10, None) == [(0, 10)]
    assert plan_chunks(10, 32) == [(0, 10)]
    assert plan_chunks(10, 4) == [(0, 4), (4, 8), (8, 10)]
    assert plan_chunks(0, 4) == []
    with pytest.raises(ValueError):
        plan_chunks(5, 0)


def test_auto_offset_budget(monkeypatch):
    from xdot.utils.env import FLAGS

    monkeypatch.setenv("XDOT_CHUNK_BUDGET_MB", "1")
    FLAGS.reload()
    try:
        o = auto_offset(10_000, 1024, torch.device("cpu"))
        assert o == (1 << 20) // 2048
        assert resolve_offset("auto", 10_000, 1024, torch.device("cpu")) == o
        assert resolve_offset("auto", 10, 1024, torch.device("cpu")) is None
    finally:
        monkeypatch.delenv("XDOT_CHUNK_BUDGET_MB")
        FLAGS.reload()
    with pytest.raises(TypeError):
        resolve_offset(2.5, 10, 1, torch.device("cpu"))


@pytest.mark.parametrize("ws", [1, 3])
def test_gather_pipeline_order_and_content(ws):
    data = torch.arange(ws * 7 * 2, dtype=torch.float32).view(ws, 7, 2)

    def body(r):
        seen = []

        def consume(s, e, g):
            assert g.shape == (ws, e - s, 2)
            assert torch.equal(g, data[:, s:e])
            seen.append((s, e))

        gather_pipeline(__import__("xdot").get_comm(), plan_chunks(7, 3), lambda s, e: data[r, s:e],
                        lambda c: (c, 2), torch.float32, torch.device("cpu"), consume)
        return seen

    res = ThreadGroup(ws).run(body)
    assert all(s == [(0, 3), (3, 6), (6, 7)] for s in res)


def test_grouped_row_gathers_keep_offset_granularity(monkeypatch):
    """nt / all with a small offset: every all-gather moves exactly one offset-row chunk (the
    reference's wire granularity), several chunks feed one GEMM per group, and at least two
    groups keep the gathers of group g+1 in flight under the GEMM of group g."""
    import xdot.parallel.functional as F
    import xdot.parallel.schedule as S
    from xdot.utils.comm import ThreadComm, ThreadGroup

    sizes, groups = [], []
    orig = ThreadComm.all_gather_into

    def spy(self, out, inp, async_op=False):
        if self.rank == 0:
            sizes.append(tuple(inp.shape))
        return orig(self, out, inp, async_op)

    monkeypatch.setattr(ThreadComm, "all_gather_into", spy)
    monkeypatch.setattr(S, "GROUP_BYTES", 7 * 3 * 2 * 6 * 8)  # 2 chunks of 3 rows per group (P=2, D=6, fp64)
    R, D, n = 10, 6, 3
    g = torch.Generator().manual_seed(0)
    L = torch.randn(2, n * R, D, generator=g, dtype=torch.float64)
    Rt = torch.randn(2, n * R, D, generator=g, dtype=torch.float64)

    def body(r):
        sl = slice(r * R, (r + 1) * R)
        orig_consume = S.gather_rows_grouped

        def wrapped(comm, r3, chunks, consume):
            def c2(s, e, gathered):
                if comm.rank == 0:
                    groups.append((s, e))
                consume(s, e, gathered)
            return orig_consume(comm, r3, chunks, c2)

        F.gather_rows_grouped = wrapped
        try:
            return F.distributed_matmul_nt(L[:, sl], Rt[:, sl], 3)
        finally:
            F.gather_rows_grouped = orig_consume

    outs = ThreadGroup(n).run(body)
    ref = L @ Rt.transpose(-1, -2)
    torch.testing.assert_close(torch.cat(outs, dim=1), ref)
    assert sizes == [(3, 2, 6)] * 3 + [(1, 2, 6)]          # (rows, P, D) per all-gather: offset rows each
    assert groups == [(0, 6), (6, 10)]                       # 2 chunks per group -> 2 GEMMs
