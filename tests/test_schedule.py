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
