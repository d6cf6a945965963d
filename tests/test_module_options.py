"""Constructor knobs of DistributedDotProductAttn beyond the reference signature:
``fused``, ``backend``, ``dtype`` (compute-dtype policy), ``chunk_plan``; plus the thread-local
backend override and its pinning into backward."""
import pytest
import torch

from xdot import DistributedDotProductAttn
from xdot import _ext


def test_fused_alias_and_validation():
    assert DistributedDotProductAttn(64, num_heads=2, fused=True).impl == "flash"
    assert DistributedDotProductAttn(64, num_heads=2, fused=False).impl == "materialized"
    with pytest.raises(ValueError):
        DistributedDotProductAttn(64, num_heads=2, fused=True, impl="materialized")
    with pytest.raises(ValueError):
        DistributedDotProductAttn(64, backend="cuda")
    with pytest.raises(ValueError):
        DistributedDotProductAttn(64, dtype=torch.int32)
    with pytest.raises(ValueError):
        DistributedDotProductAttn(64, chunk_plan=0)
    m = DistributedDotProductAttn(64, num_heads=2, backend="torch", dtype=torch.bfloat16, chunk_plan=2)
    r = repr(m)
    assert "backend=torch" in r and "chunk_plan=2" in r and "bfloat16" in r


def test_backend_override_scopes_and_pins():
    assert _ext.current_backend() in ("auto", "hip", "torch")
    with _ext.backend("torch"):
        assert _ext.current_backend() == "torch"
        with _ext.backend(None):  # None / 'auto' keep the enclosing choice
            assert _ext.current_backend() == "torch"
    assert _ext.current_backend() != "torch" or _ext.FLAGS.backend == "torch"
    with pytest.raises(ValueError):
        _ext.backend("cuda")

    seen = {}

    class F(torch.autograd.Function):
        @staticmethod
        @_ext.pinned
        def forward(ctx, x):
            return x * 2

        @staticmethod
        @_ext.pinned
        def backward(ctx, g):
            seen["bwd"] = _ext.current_backend()
            return g * 2

    x = torch.ones(3, requires_grad=True)
    with _ext.backend("torch"):
        y = F.apply(x)
    y.sum().backward()  # outside the context: backward still sees 'torch'
    assert seen["bwd"] == "torch"
    torch.testing.assert_close(x.grad, torch.full((3,), 2.0))


@pytest.mark.parametrize("impl", ["materialized", "flash", "ring"])
def test_compute_dtype_policy(impl):
    """fp32 master params + inputs, bf16 compute: equals running a bf16 copy of the module,
    output comes back in fp32, gradients land on the fp32 parameters."""
    torch.manual_seed(0)
    m = DistributedDotProductAttn(64, num_heads=4, dtype=torch.bfloat16, impl=impl)
    ref = DistributedDotProductAttn(64, num_heads=4, impl=impl).to(torch.bfloat16)
    ref.load_state_dict({k: v.to(torch.bfloat16) for k, v in m.state_dict().items()})
    x = torch.rand(1, 24, 64)
    mask = torch.rand(1, 24, 24) < 0.2
    mask[..., 0] = False
    out = m(x, x, x, mask)
    assert out.dtype == torch.float32
    out_ref = ref(x.to(torch.bfloat16), x.to(torch.bfloat16), x.to(torch.bfloat16), mask)
    torch.testing.assert_close(out, out_ref.float(), atol=0, rtol=0)
    out.sum().backward()
    out_ref.float().sum().backward()
    for (n, p), (_, q) in zip(m.named_parameters(), ref.named_parameters()):
        assert p.dtype == torch.float32 and p.grad is not None and p.grad.dtype == torch.float32, n
        torch.testing.assert_close(p.grad, q.grad.float(), atol=2e-2, rtol=2e-2)


def test_packed_qv_parameters_share_storage():
    """queries / values weights live in ONE storage after the first forward (the packed [q|v]
    weight is a view, no per-step cat); state_dict keys, .to() and load_state_dict keep working
    (a .to() re-packs on the next forward) and the gradients match the unpacked materialised path."""
    import copy

    from xdot import DistributedDotProductAttn
    from xdot.models.attention import _adjacent

    torch.manual_seed(0)
    m = DistributedDotProductAttn(32, num_heads=4, add_bias=True, impl="flash", distributed=False).double()
    ref = copy.deepcopy(m)
    ref.impl = "materialized"  # separate q / v projections, no packing
    x = torch.randn(1, 7, 32, dtype=torch.float64)
    out = m(x, x, x, None)
    assert _adjacent(m.queries.weight, m.values.weight) and _adjacent(m.queries.bias, m.values.bias)
    assert not _adjacent(ref.queries.weight, ref.values.weight)
    out.square().sum().backward()
    ref(x, x, x, None).square().sum().backward()
    for (n, p), (_, q) in zip(m.named_parameters(), ref.named_parameters()):
        if n == "queries.bias":
            continue  # exactly zero up to rounding (softmax shift invariance)
        torch.testing.assert_close(p.grad, q.grad, rtol=1e-9, atol=1e-11, msg=n)
    m2 = m.to(torch.float32)
    x32 = x.float()
    m2(x32, x32, x32, None)
    assert _adjacent(m2.queries.weight, m2.values.weight)
    sd = m2.state_dict()
    assert {"queries.weight", "values.weight", "queries.bias", "values.bias"} <= set(sd)
    m2.load_state_dict(sd)
    assert _adjacent(m2.queries.weight, m2.values.weight)


def test_library_weight_gradient_stays_on_current_stream():
    """A weight gradient that falls back to a library GEMM (fp32 / fp64, CPU) ignores the
    ``_xdot_ready_on`` side-stream hint: two library GEMMs in flight on two streams can deadlock
    (stream-K kernels spinning on each other's unscheduled workgroups), so only the xdot MFMA
    weight gradient may run beside other work (``xdot.ops.linear.native_wgrad``)."""
    from xdot.ops.linear import linear_backward, native_wgrad

    x = torch.randn(6, 5, dtype=torch.float64)
    w = torch.randn(4, 5, dtype=torch.float64)
    dy = torch.randn(6, 4, dtype=torch.float64)
    assert not native_wgrad(dy, x) and not native_wgrad(dy.float(), x.float())
    dy._xdot_ready_on = object()  # would fail as a stream context if it were used
    dx, dw, db = linear_backward(dy, x, w, True, True, True)
    torch.testing.assert_close(dx, dy @ w)
    torch.testing.assert_close(dw, dy.t() @ x)
    torch.testing.assert_close(db, dy.sum(0))


def test_weight_grad_pair_and_prescale_gate_cpu():
    """CPU tensors: weight_grad_pair falls back to two weight_grad products (dyᵀ·x, fp32
    accumulation, cast to the requested dtype) and the row pre-scale is never wanted."""
    from xdot.ops.linear import weight_grad_pair
    from xdot.parallel.attention import prescale_wanted

    g = torch.Generator().manual_seed(3)
    dy0, x0 = torch.randn(2, 5, 128, generator=g), torch.randn(2, 5, 256, generator=g)
    dy1, x1 = torch.randn(10, 256, generator=g), torch.randn(10, 128, generator=g)
    a, b = weight_grad_pair(dy0, x0, dy1, x1, torch.float32)
    torch.testing.assert_close(a, dy0.reshape(-1, 128).t() @ x0.reshape(-1, 256), rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(b, dy1.t() @ x1, rtol=1e-5, atol=1e-5)
    assert a.shape == (128, 256) and b.shape == (256, 128)
    k = torch.randn(1, 16, 64, dtype=torch.bfloat16)
    assert not prescale_wanted(k, torch.cat([k, k], -1), 4)
