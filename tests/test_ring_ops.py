"""Ring schedule of the distributed products (``schedule='ring'`` / ``XDOT_OPS_SCHEDULE=ring``):
point-to-point hops instead of all-gather / reduce-scatter must give the same results as the
gather schedule and the dense product (CPU ranks, float64, world sizes 2-4, 3-D and 4-D
operands), including the autograd ops whose backward reuses the schedule."""
import pytest
import torch

from xdot.utils.comm import ThreadGroup


def _full(seed, ws, P, R, D):
    g = torch.Generator().manual_seed(seed)
    T = R * ws
    A = torch.randn(*P, T, D, generator=g, dtype=torch.float64)
    B = torch.randn(*P, T, D, generator=g, dtype=torch.float64)
    S = torch.randn(*P, T, T, generator=g, dtype=torch.float64)
    return A, B, S


def _rank_case(rank, ws, P, R, D, seed):
    from xdot.parallel import distributed_matmul_all, distributed_matmul_nt, distributed_matmul_tn

    A, B, S = _full(seed, ws, P, R, D)
    sl = slice(rank * R, (rank + 1) * R)
    a, b, s = A[..., sl, :], B[..., sl, :], S[..., sl, :]
    for sched in ("ring", "gather"):
        nt = distributed_matmul_nt(a, b, schedule=sched, alpha=0.5)
        torch.testing.assert_close(nt, 0.5 * (A @ B.transpose(-1, -2))[..., sl, :], rtol=1e-12, atol=1e-10)
        al = distributed_matmul_all(s, b, schedule=sched)
        torch.testing.assert_close(al, (S @ B)[..., sl, :], rtol=1e-12, atol=1e-10)
        tn = distributed_matmul_tn(s, b, schedule=sched)
        torch.testing.assert_close(tn, (S.transpose(-1, -2) @ B)[..., sl, :], rtol=1e-12, atol=1e-10)


@pytest.mark.parametrize("ws", [2, 3, 4])
@pytest.mark.parametrize("P", [(), (2,), (2, 3)])
def test_ring_products_match_dense(ws, P):
    ThreadGroup(ws).run(lambda r: _rank_case(r, ws, P, 5, 7, 11))


def _autograd_case(rank, ws):
    import os

    from xdot.parallel import FullMultiplication, LeftTransposeMultiplication, RightTransposeMultiplication
    from xdot.utils.env import FLAGS

    R, D = 4, 6
    A, B, S = _full(3, ws, (2,), R, D)
    sl = slice(rank * R, (rank + 1) * R)
    grads = {}
    for sched in ("ring", "gather"):
        FLAGS.ops_schedule = sched
        a = A[..., sl, :].clone().requires_grad_(True)
        b = B[..., sl, :].clone().requires_grad_(True)
        s = S[..., sl, :].clone().requires_grad_(True)
        y = (RightTransposeMultiplication.apply(a, b, None).square().sum()
             + FullMultiplication.apply(s, b, None).square().sum()
             + LeftTransposeMultiplication.apply(s, a, None).square().sum())
        y.backward()
        grads[sched] = (a.grad, b.grad, s.grad)
    FLAGS.reload()
    for x, y_ in zip(grads["ring"], grads["gather"]):
        torch.testing.assert_close(x, y_, rtol=1e-11, atol=1e-10)


@pytest.mark.parametrize("ws", [2, 3])
def test_ring_schedule_autograd_ops(ws):
    ThreadGroup(ws).run(lambda r: _autograd_case(r, ws))


def test_schedule_validation():
    from xdot.parallel import distributed_matmul_nt

    with pytest.raises(ValueError):
        distributed_matmul_nt(torch.randn(2, 3), torch.randn(2, 3), schedule="tree")
