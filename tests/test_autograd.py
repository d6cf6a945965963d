"""Autograd correctness of the three distributed multiplication ops (float64 gradcheck).

The reference never tests its autograd ops directly, and its LeftTransposeMultiplication
returns a transposed left gradient (reference ``multiplication/ops.py:69``).  Here every op
is checked against autograd of the dense product on the gathered tensors, for several world
sizes and offsets, through in-process ranks.
"""
import pytest
import torch

from xdot.utils.comm import ThreadGroup

WS_CASES = [1, 2, 3]


def _shard(x, r, ws):
    R = x.shape[-2] // ws
    return x[..., r * R:(r + 1) * R, :].detach().clone().requires_grad_(True)


def _check(op_name, ws, offset, compat=False):
    import xdot.parallel.autograd as A
    import xdot.parallel.functional as F

    R, D = 3, 4
    T = ws * R
    g = torch.Generator().manual_seed(1)
    if op_name == "RightTranspose":
        L, Rg = torch.randn(2, T, D, generator=g, dtype=torch.float64), torch.randn(2, T, D, generator=g, dtype=torch.float64)
        dense = lambda a, b: a @ b.transpose(-1, -2)  # noqa: E731
        op = A.RightTransposeMultiplication
    elif op_name == "Full":
        L, Rg = torch.randn(2, T, T, generator=g, dtype=torch.float64), torch.randn(2, T, D, generator=g, dtype=torch.float64)
        dense = lambda a, b: a @ b  # noqa: E731
        op = A.FullMultiplication
    else:
        L, Rg = torch.randn(2, T, T, generator=g, dtype=torch.float64), torch.randn(2, T, D, generator=g, dtype=torch.float64)
        dense = lambda a, b: a.transpose(-1, -2) @ b  # noqa: E731
        op = A.LeftTransposeMultiplication
    W = torch.randn(dense(L, Rg).shape, generator=g, dtype=torch.float64)

    Lf, Rf = L.clone().requires_grad_(True), Rg.clone().requires_grad_(True)
    (dense(Lf, Rf) * W).sum().backward()

    def body(r):
        l, rr = _shard(L, r, ws), _shard(Rg, r, ws)
        out = op.apply(l, rr, offset)
        w = W[..., r * R:(r + 1) * R, :]
        (out * w).sum().backward()
        gl = F.gather_sequence(l.grad, -2)
        gr = F.gather_sequence(rr.grad, -2)
        return gl, gr

    prev = A.LeftTransposeMultiplication.compat_reference_bug
    A.LeftTransposeMultiplication.compat_reference_bug = compat
    try:
        gl, gr = ThreadGroup(ws).run(body)[0]
    finally:
        A.LeftTransposeMultiplication.compat_reference_bug = prev
    return gl, gr, Lf.grad, Rf.grad


@pytest.mark.parametrize("ws", WS_CASES)
@pytest.mark.parametrize("op_name", ["RightTranspose", "Full", "LeftTranspose"])
@pytest.mark.parametrize("offset", [None, 2])
def test_op_gradients(op_name, ws, offset):
    gl, gr, rl, rr = _check(op_name, ws, offset)
    torch.testing.assert_close(gl, rl)
    torch.testing.assert_close(gr, rr)


def test_left_transpose_reference_bug_flag():
    """compat flag reproduces the reference's transposed block (only meaningful when R == T)."""
    gl, gr, rl, rr = _check("LeftTranspose", 1, None, compat=True)
    torch.testing.assert_close(gl, rl.transpose(-1, -2))
    torch.testing.assert_close(gr, rr)


@pytest.mark.parametrize("ws", [1, 2])
def test_gradcheck_single_process(ws):
    """torch.autograd.gradcheck through the ops (ws=1 uses LocalComm, ws=2 threads)."""
    import xdot.parallel.autograd as A

    if ws == 1:
        a = torch.randn(2, 3, 4, dtype=torch.float64, requires_grad=True)
        b = torch.randn(2, 3, 4, dtype=torch.float64, requires_grad=True)
        s = torch.randn(2, 3, 3, dtype=torch.float64, requires_grad=True)
        assert torch.autograd.gradcheck(lambda x, y: A.RightTransposeMultiplication.apply(x, y, 2), (a, b))
        assert torch.autograd.gradcheck(lambda x, y: A.FullMultiplication.apply(x, y, 1), (s, b))
        assert torch.autograd.gradcheck(lambda x, y: A.LeftTransposeMultiplication.apply(x, y, 1), (s, b))
    else:
        for name in ("RightTranspose", "Full", "LeftTranspose"):
            gl, gr, rl, rr = _check(name, ws, 1)
            torch.testing.assert_close(gl, rl)
            torch.testing.assert_close(gr, rr)
