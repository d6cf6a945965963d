"""Segmented multi-rank forward of the fused path (local block first, then each gathered
chunk's peer blocks, one log-sum-exp combine): CPU ranks, float64, against the single-device
module.  Covers rows that one segment masks entirely (own block or a whole peer block), the
chunked gather plan, and the XDOT_LOCAL_FIRST=0 schedule."""
import pytest
import torch

D, H, L = 32, 4, 10  # L rows per rank (not a multiple of the chunk count)


def _case(rank, ws, chunks, local_first, seed):
    from xdot import DistributedDotProductAttn
    from xdot.parallel import gather_sequence
    from xdot.parallel.attention import seq_parallel_attention_packed, start_gather
    from xdot.utils.env import FLAGS

    FLAGS.local_first = local_first
    torch.manual_seed(0)
    T = L * ws
    g = torch.Generator().manual_seed(seed)
    k_full = torch.randn(1, T, D, generator=g, dtype=torch.float64)
    qv_full = torch.randn(1, T, 2 * D, generator=g, dtype=torch.float64)
    mask = torch.rand(1, T, T, generator=g) < 0.3
    mask[:, :L, :L] = True                 # rank 0's rows: own block fully masked
    mask[:, L:2 * L, :] = True             # rank 1's rows: everything but column 0 masked
    mask[:, L:2 * L, 0] = False
    mask[..., torch.arange(T), torch.arange(T)] &= torch.arange(T) >= 2 * L  # keep a live column per row
    mask[:, :L, L] = False
    sl = slice(rank * L, (rank + 1) * L)
    k = k_full[:, sl].clone().requires_grad_(True)
    qv = qv_full[:, sl].clone().requires_grad_(True)
    pend = start_gather(qv, chunks=chunks)
    assert len(pend.chunks) == min(chunks, L)
    o = seq_parallel_attention_packed(k, qv, mask[:, sl], H, 0.3, pending=pend)
    o.square().sum().backward()

    kf = k_full.clone().requires_grad_(True)
    qvf = qv_full.clone().requires_grad_(True)
    kh = kf.view(1, T, H, D // H).transpose(1, 2)
    qh = qvf[..., :D].reshape(1, T, H, D // H).transpose(1, 2)
    vh = qvf[..., D:].reshape(1, T, H, D // H).transpose(1, 2)
    s = (kh @ qh.transpose(-1, -2) * 0.3).masked_fill(mask.unsqueeze(1), -float("inf"))
    ref = (s.softmax(-1) @ vh).transpose(1, 2).reshape(1, T, D)
    ref.square().sum().backward()
    torch.testing.assert_close(gather_sequence(o.detach(), -2), ref.detach(), atol=1e-10, rtol=1e-10)
    torch.testing.assert_close(gather_sequence(k.grad, -2), kf.grad, atol=1e-9, rtol=1e-9)
    torch.testing.assert_close(gather_sequence(qv.grad, -2), qvf.grad, atol=1e-9, rtol=1e-9)
    FLAGS.reload()


@pytest.mark.parametrize("ws", [2, 3])
@pytest.mark.parametrize("chunks", [1, 2, 3])
@pytest.mark.parametrize("local_first", [True, False])
def test_segmented_forward_threads(ws, chunks, local_first):
    from xdot.utils.comm import ThreadGroup

    ThreadGroup(ws).run(lambda r: _case(r, ws, chunks, local_first, 5))


def test_segment_plan_skips_own_rank():
    from xdot.parallel.attention import _segment_plan

    assert _segment_plan(4, 0, 1, True) == [(0, 1, 4)]
    assert _segment_plan(4, 3, 2, True) == [(0, 0, 3), (1, 0, 3)]
    assert _segment_plan(4, 1, 1, True) == [(0, 0, 1), (0, 2, 4)]
    assert _segment_plan(4, 1, 2, False) == [(0, 0, 4), (1, 0, 4)]


def _gpu_case(rank, ws, chunks, local_first):
    import os

    from xdot.parallel import gather_sequence
    from xdot.parallel.attention import _hip_ok, seq_parallel_attention_packed, start_gather
    from xdot.utils.env import FLAGS

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    os.environ["XDOT_LOCAL_FIRST"] = "1" if local_first else "0"
    FLAGS.reload()
    Dg, Hg, Lg = 256, 4, 200
    T = Lg * ws
    g = torch.Generator().manual_seed(9)
    k_full = torch.randn(1, T, Dg, generator=g).to(dev, torch.bfloat16)
    qv_full = torch.randn(1, T, 2 * Dg, generator=g).to(dev, torch.bfloat16)
    mask = torch.rand(1, T, T, generator=g) < 0.3
    mask[:, :Lg, :Lg] = True                        # rank 0's rows: own block fully masked
    mask[:, :Lg, Lg] = False
    mask = mask.to(dev)
    sl = slice(rank * Lg, (rank + 1) * Lg)
    k = k_full[:, sl].clone().requires_grad_(True)
    qv = qv_full[:, sl].clone().requires_grad_(True)
    assert _hip_ok(k, qv, Hg)
    pend = start_gather(qv, chunks=chunks)
    o = seq_parallel_attention_packed(k, qv, mask[:, sl], Hg, 0.125, pending=pend)
    o.float().square().sum().backward()

    kf = k_full.float().requires_grad_(True)
    qvf = qv_full.float().requires_grad_(True)
    kh = kf.view(1, T, Hg, Dg // Hg).transpose(1, 2)
    qh = qvf[..., :Dg].reshape(1, T, Hg, Dg // Hg).transpose(1, 2)
    vh = qvf[..., Dg:].reshape(1, T, Hg, Dg // Hg).transpose(1, 2)
    s = (kh @ qh.transpose(-1, -2) * 0.125).masked_fill(mask.unsqueeze(1), -float("inf"))
    ref = (s.softmax(-1) @ vh).transpose(1, 2).reshape(1, T, Dg)
    ref.square().sum().backward()

    def rel(a, b):
        return ((a.float() - b.float()).norm() / b.float().norm()).item()

    assert rel(gather_sequence(o.detach(), -2), ref) <= 1e-2
    assert rel(gather_sequence(k.grad, -2), kf.grad) <= 2e-2
    assert rel(gather_sequence(qv.grad, -2), qvf.grad) <= 2e-2


@pytest.mark.gpu
@pytest.mark.parametrize("chunks,local_first", [(1, True), (2, True), (3, True), (2, False)])
def test_segmented_forward_gpu(gpu, chunks, local_first):
    """The HIP segment kernels + combine, 3 gloo ranks sharing the GPU (the autograd engine
    runs every CUDA backward of a process on one device thread, so in-process ranks would
    deadlock in the backward's collective)."""
    from _dist import run_gloo

    run_gloo(_gpu_case, 3, chunks, local_first, timeout=400)
