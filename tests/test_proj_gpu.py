"""Projection GEMM (``csrc/gemm_proj.hip``, ``torch.ops.xdot.proj``) against a plain PyTorch fp32
reference of the same product: the module's Linear forward ``x Wᵀ + b`` (NT) and input gradient
``dy W`` (NN) at the per-rank shapes (T/N = 3125 and 25000 rows, 768 / 1536 features), odd row
counts, every tile configuration, leading batch dims, an output view inside a larger buffer (the
all-gather slot), and the module-level route (forward + backward through ``LinearFn``)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

dev = torch.device("cuda", 0) if torch.cuda.is_available() else None


def _ops():
    import xdot._ext as ext

    assert ext.load(), "xdot/_C.so missing"
    return ext.ops()


def _check(got, ref, dt):
    ref32 = ref.float()
    err = (got.float() - ref32).abs().max().item()
    tol = (2e-2 if dt == torch.bfloat16 else 4e-3) * max(1.0, ref32.abs().max().item())
    assert err <= tol, f"max abs err {err} > {tol}"
    rel = ((got.float() - ref32).norm() / ref32.norm().clamp_min(1e-30)).item()
    assert rel < (4e-3 if dt == torch.bfloat16 else 6e-4), rel


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("M,N,K", [(3125, 1536, 768), (3125, 768, 768), (25000, 1536, 768), (1, 64, 64),
                                   (7, 128, 128), (100, 192, 64), (129, 256, 1536), (4000, 768, 1536)])
@pytest.mark.parametrize("bias", [False, True])
def test_proj_nt(dt, M, N, K, bias):
    torch.manual_seed(M + N + K)
    x = torch.randn(M, K, device=dev, dtype=dt)
    w = torch.randn(N, K, device=dev, dtype=dt) / K ** 0.5
    b = torch.randn(N, device=dev, dtype=dt) if bias else None
    y = _ops().proj(x, w, b, False, None, 1)  # force: the kernel at every size
    ref = x.float() @ w.float().t() + (b.float() if bias else 0.0)
    assert y.shape == (M, N) and y.dtype == dt
    _check(y, ref, dt)


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("M,Nout,Nin", [(3125, 1536, 768), (3125, 768, 768), (25000, 768, 768), (1, 64, 128),
                                        (77, 192, 256), (3125, 768, 1536)])
def test_proj_nn(dt, M, Nout, Nin):
    torch.manual_seed(M + Nout)
    dy = torch.randn(M, Nout, device=dev, dtype=dt)
    w = torch.randn(Nout, Nin, device=dev, dtype=dt) / Nout ** 0.5
    dx = _ops().proj(dy, w, None, True, None, 1)
    assert dx.shape == (M, Nin)
    _check(dx, dy.float() @ w.float(), dt)


def test_proj_batched_strided_and_out_view():
    """(B, R, K) input, weight rows from a packed parameter (row-stride view), output written into
    rank 2's block of an (n, B, R, N) gather buffer; the other blocks are untouched."""
    dt = torch.bfloat16
    torch.manual_seed(0)
    x = torch.randn(1, 3125, 768, device=dev, dtype=dt)
    packed = torch.randn(2 * 768, 768, device=dev, dtype=dt) / 28.0
    w = packed[768:]  # the values half of a [q|v] weight
    b = torch.randn(1536, device=dev, dtype=dt)[768:]
    y = _ops().proj(x, w, b, False, None, 1)
    assert y.shape == (1, 3125, 768)
    ref = x.float() @ w.float().t() + b.float()
    _check(y, ref, dt)
    gbuf = torch.full((4, 1, 3125, 768), 7.0, device=dev, dtype=dt)
    _ops().proj(x, w, b, False, gbuf[2].view(-1, 768), 1)
    _check(gbuf[2], ref, dt)
    for r in (0, 1, 3):
        assert torch.all(gbuf[r] == 7.0)


def test_proj_fallback_shapes_match_library():
    """Shapes outside the kernel's envelope (K % 64, N % 64, fp32) and, unforced, the products
    large enough for hipBLASLt to be faster take the library route in the same op and still
    match the reference."""
    torch.manual_seed(1)
    for dt, M, N, K in [(torch.bfloat16, 50, 96, 100), (torch.bfloat16, 50, 100, 64), (torch.float32, 64, 128, 64),
                        (torch.bfloat16, 25000, 1536, 768)]:
        x = torch.randn(M, K, device=dev, dtype=dt)
        w = torch.randn(N, K, device=dev, dtype=dt) / K ** 0.5
        _check(_ops().proj(x, w, None, False, None), x.float() @ w.float().t(), dt if dt != torch.float32 else torch.float16)


def test_linear_fn_routes_through_proj():
    """xdot.ops.linear.linear forward / backward vs torch autograd on the same fp32 math."""
    from xdot.ops.linear import linear

    dt = torch.bfloat16
    torch.manual_seed(2)
    x = torch.randn(2, 700, 768, device=dev, dtype=dt, requires_grad=True)
    w = (torch.randn(1536, 768, device=dev, dtype=dt) / 28.0).requires_grad_()
    b = torch.randn(1536, device=dev, dtype=dt, requires_grad=True)
    y = linear(x, w, b)
    g = torch.randn_like(y)
    y.backward(g)
    xr, wr, br = (t.detach().float().requires_grad_() for t in (x, w, b))
    yr = torch.nn.functional.linear(xr, wr, br)
    yr.backward(g.float())
    _check(y.detach(), yr.detach(), dt)
    _check(x.grad, xr.grad, dt)
    _check(w.grad, wr.grad, dt)
    _check(b.grad, br.grad, dt)


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("K,M,N,S", [(3125, 768, 768, 0), (3125, 1536, 768, 0), (25000, 768, 768, 0), (100, 128, 256, 0),
                                     (64, 128, 128, 0), (1, 128, 128, 0), (129, 256, 128, 3), (3125, 768, 768, 49)])
def test_wgrad(dt, K, M, N, S):
    """Weight-gradient kernel (csrc/gemm_wgrad.hip) dyᵀ·x vs fp32 torch: K slabs with a partial last
    k-tile (zeros past K through the buffer descriptor), one slab per k-tile, fp32 and 16-bit
    outputs."""
    torch.manual_seed(K + M + N)
    dy = torch.randn(K, M, device=dev, dtype=dt)
    x = torch.randn(K, N, device=dev, dtype=dt)
    ref = dy.float().t() @ x.float()
    for odt in (dt, torch.float32):
        got = _ops().wgrad(dy, x, odt, S)
        assert got is not None and got.shape == (M, N) and got.dtype == odt
        _check(got, ref, dt)


def test_wgrad_declines_and_weight_grad_routes():
    """Shapes the kernel does not take come back undefined; xdot.ops.linear.weight_grad then runs
    the gemm3 / slab routes with the same result."""
    from xdot.ops.linear import weight_grad

    dt = torch.bfloat16
    dy = torch.randn(500, 96, device=dev, dtype=dt)
    x = torch.randn(500, 128, device=dev, dtype=dt)
    assert _ops().wgrad(dy, x, dt, 0) is None
    _check(weight_grad(dy, x), dy.float().t() @ x.float(), dt)
    dy = torch.randn(3125, 768, device=dev, dtype=dt)
    x = torch.randn(3125, 768, device=dev, dtype=dt)
    _check(weight_grad(dy, x), dy.float().t() @ x.float(), dt)


@pytest.mark.parametrize("M,force", [(3125, 1), (25000, 0), (100, 1)])
@pytest.mark.parametrize("bias", [False, True])
def test_proj_alpha(M, force, bias):
    """C = alpha (x Wᵀ + b) rounded once, on the kernel (force) and on the library route (the
    fused module folds the attention's row pre-scale into the k projection this way)."""
    dt = torch.bfloat16
    torch.manual_seed(M)
    x = torch.randn(M, 768, device=dev, dtype=dt)
    w = torch.randn(768, 768, device=dev, dtype=dt) / 28.0
    b = torch.randn(768, device=dev, dtype=dt) if bias else None
    alpha = 0.036084391824351615 * 1.4426950408889634  # 1/sqrt(768) * log2 e
    y = _ops().proj(x, w, b, False, None, force, alpha)
    ref = alpha * (x.float() @ w.float().t() + (b.float() if bias else 0.0))
    _check(y, ref, dt)


@pytest.mark.parametrize("K", [3125, 25000, 100])
def test_wgrad_pair_one_launch(K):
    """Two weight gradients in one launch (the fused backward's dWk and dW[q|v]) equal the
    separate products (bitwise: same slabs, same ordered sums)."""
    from xdot.ops.linear import weight_grad_pair

    dt = torch.bfloat16
    torch.manual_seed(K)
    x = torch.randn(K, 768, device=dev, dtype=dt)
    dk = torch.randn(K, 768, device=dev, dtype=dt)
    dqv = torch.randn(K, 1536, device=dev, dtype=dt)
    outs = _ops().wgrad2(dk, x, dqv, x, dt)
    assert len(outs) == 2
    assert torch.equal(outs[0], _ops().wgrad(dk, x, dt, 0)) and torch.equal(outs[1], _ops().wgrad(dqv, x, dt, 0))
    _check(outs[1], dqv.float().t() @ x.float(), dt)
    a, b = weight_grad_pair(dk.view(1, K, 768), x.view(1, K, 768), dqv.view(1, K, 1536), x.view(1, K, 768))
    assert torch.equal(a, outs[0]) and torch.equal(b, outs[1])
    assert _ops().wgrad2(dk[:, :96], x, dqv, x, dt) == []  # not eligible: the caller falls back
