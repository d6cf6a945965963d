"""Operator parity of the distributed products (CPU; gloo processes and in-process ranks).

Mirrors the reference's operator suite (``tests/test_multiplication.py``: six modes NT, NT-4D,
TN, TN-4D, FULL, FULL-4D on integer ``arange`` tensors compared with ``==``, offset=2) and
extends it: world sizes 1-4, offsets that do not divide the shard (short last chunk),
``offset=None``/``'auto'``, float dtypes with tolerances.
"""
import functools

import pytest
import torch

from _dist import run_gloo

ROWS = 4   # rows per rank (reference LENGTH)
DIM = 6    # feature dim (reference DIM)


def arange(*shape, dtype=torch.int64):
    n = functools.reduce(lambda a, b: a * b, shape)
    return torch.arange(n, dtype=dtype).view(*shape)


def heads_layout(T, D, H=2):
    """(1, H, T, D/H) multi-head layout of a (1, T, D) arange tensor."""
    return arange(1, T, D).view(1, T, H, D // H).transpose(1, 2).contiguous()


def shard(x, rank, ws, dim=-2):
    R = x.shape[dim] // ws
    return x.narrow(dim % x.dim(), rank * R, R).contiguous()


def cases(ws):
    T = ROWS * ws
    return {
        "NT": (arange(1, T, DIM), arange(1, T, DIM), lambda a, b: a @ b.transpose(-1, -2), "nt"),
        "NT-4D": (heads_layout(T, DIM), heads_layout(T, DIM), lambda a, b: a @ b.transpose(-1, -2), "nt"),
        "TN": (arange(1, T, T), arange(1, T, DIM), lambda a, b: a.transpose(-1, -2) @ b, "tn"),
        "TN-4D": (arange(1, 2, T, T), heads_layout(T, DIM), lambda a, b: a.transpose(-1, -2) @ b, "tn"),
        "FULL": (arange(1, T, T), arange(1, T, DIM), lambda a, b: a @ b, "all"),
        "FULL-4D": (arange(1, 2, T, T), heads_layout(T, DIM), lambda a, b: a @ b, "all"),
    }


def run_case(op, left, right, offset, chunking="rows"):
    import xdot.parallel.functional as F

    if op == "nt":
        return F.distributed_matmul_nt(left, right, offset)
    if op == "all":
        return F.distributed_matmul_all(left, right, offset, chunking=chunking)
    return F.distributed_matmul_tn(left, right)


def check_all_modes(rank, ws, offsets):
    import xdot.parallel.functional as F

    for name, (gl, gr, gt_fn, op) in cases(ws).items():
        gt = gt_fn(gl, gr)
        for off in offsets:
            # distributed_matmul_all: the default row-block plan and the reference's literal
            # feature-column plan (same per-step gather budget)
            for chunking in (("rows", "columns") if op == "all" else ("rows",)):
                res = run_case(op, shard(gl, rank, ws), shard(gr, rank, ws), off, chunking)
                full = F.gather_sequence(res, -2)
                assert full.shape == gt.shape, (name, off, full.shape, gt.shape)
                assert torch.equal(full, gt), f"{name} offset={off} chunking={chunking} rank={rank}"


@pytest.mark.parametrize("ws", [1, 2, 3])
def test_modes_gloo(ws):
    run_gloo(check_all_modes, ws, [2, 3, None])


@pytest.mark.parametrize("ws", [1, 2, 4])
def test_modes_threads(ws):
    from xdot.utils.comm import ThreadGroup

    ThreadGroup(ws).run(lambda r: check_all_modes(r, ws, [1, 2, 3, 5, None, "auto"]))


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64, torch.bfloat16])
def test_float_dtypes_threads(dtype):
    from xdot.utils.comm import ThreadGroup
    import xdot.parallel.functional as F

    ws, R, D = 3, 5, 8
    T = ws * R
    g = torch.Generator().manual_seed(0)
    A = torch.randn(2, T, D, generator=g)
    Bm = torch.randn(2, T, D, generator=g)
    S = torch.randn(2, T, T, generator=g)
    tol = dict(atol=5e-2, rtol=5e-2) if dtype == torch.bfloat16 else dict(atol=1e-5, rtol=1e-5)

    def body(r):
        a, b, s = (shard(x, r, ws).to(dtype) for x in (A, Bm, S))
        nt = F.gather_sequence(F.distributed_matmul_nt(a, b, 2), -2)
        al = F.gather_sequence(F.distributed_matmul_all(s, b, 3), -2)
        tn = F.gather_sequence(F.distributed_matmul_tn(s, b), -2)
        assert nt.dtype == dtype and al.dtype == dtype and tn.dtype == dtype
        Ad, Bd, Sd = A.to(dtype).double(), Bm.to(dtype).double(), S.to(dtype).double()
        torch.testing.assert_close(nt.double(), Ad @ Bd.transpose(-1, -2), **tol)
        torch.testing.assert_close(al.double(), Sd @ Bd, **tol)
        torch.testing.assert_close(tn.double(), Sd.transpose(-1, -2) @ Bd, **tol)

    ThreadGroup(ws).run(body)


def test_nt_alpha_and_out_dtype():
    import xdot.parallel.functional as F

    a = torch.randn(3, 4, 5)
    b = torch.randn(3, 4, 5)
    r = F.distributed_matmul_nt(a, b, alpha=0.5, out_dtype=torch.float64)
    assert r.dtype == torch.float64
    torch.testing.assert_close(r, (0.5 * a @ b.transpose(-1, -2)).double())


def test_block_sum_allreduce_threads():
    from xdot.utils.comm import ThreadGroup
    import xdot.parallel.functional as F

    ws = 3
    L = [torch.randn(2, 4, 5) for _ in range(ws)]
    Rm = [torch.randn(2, 5, 3) for _ in range(ws)]
    ref = sum(l @ r for l, r in zip(L, Rm))

    def body(r):
        out = F.distributed_matmul_block(L[r], Rm[r])
        torch.testing.assert_close(out, ref)
        outT = F.distributed_matmul_block(L[r], Rm[r], transpose=True)
        torch.testing.assert_close(outT, ref.transpose(-1, -2))

    ThreadGroup(ws).run(body)


def test_shape_errors():
    import xdot.parallel.functional as F

    with pytest.raises(ValueError):
        F.distributed_matmul_nt(torch.zeros(2, 3, 4), torch.zeros(3, 3, 4))
    with pytest.raises(ValueError):
        F.distributed_matmul_all(torch.zeros(1, 3, 5), torch.zeros(1, 3, 4))
    with pytest.raises(ValueError):
        F.distributed_matmul_nt(torch.zeros(1, 3, 4), torch.zeros(1, 3, 4), offset=0)
