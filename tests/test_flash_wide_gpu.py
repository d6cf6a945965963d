"""Wide-head flash kernels (csrc/flash_wide.hip, D = 160 / 192 / 256 / 384) vs an fp64 PyTorch
reference (GPU only).  The reference's own configurations need them: example.py:20 (768 features,
2 heads: D = 384) and tests/test_gradient.py:45 (num_heads = 1 at 256 features: D = 256).

bf16 is bounded like the narrow bf16 kernels (relative Frobenius <= 2e-2); exact fp32 like
flash_f32 (<= 2e-6; fp32 D = 384 runs on the score buffer, D <= 256 both ways)."""
import math

import pytest
import torch

from test_flash_f32_gpu import _ref64, _rel
from test_flash_gpu import _to_gathered

pytestmark = pytest.mark.gpu

WIDE_CASES = [
    # (B, R, N, Rc, H, D)
    (1, 200, 1, 300, 2, 384),
    (1, 150, 2, 100, 1, 256),
    (2, 130, 1, 97, 2, 192),
    (1, 77, 3, 50, 3, 160),
]


def _inputs(case, mask_kind, gpu, dtype):
    B, R, N, Rc, H, D = case
    C, T = H * D, N * Rc
    g = torch.Generator(device="cpu").manual_seed(sum(case) + 3)
    rows = torch.randn(B, R, C, generator=g).to(gpu, dtype)
    kc = torch.randn(N, B, Rc, C, generator=g).to(gpu, dtype)
    vc = torch.randn(N, B, Rc, C, generator=g).to(gpu, dtype)
    do = torch.randn(B, R, C, generator=g).to(gpu, dtype)
    mask = None
    if mask_kind == "random":
        mask = torch.rand(B, R, T, generator=g) < 0.4
    elif mask_kind == "blocks":
        mask = torch.zeros(B, R, T, dtype=torch.bool)
        mask[:, :, : min(T, 64)] = True
        r1 = min(R, 90)
        mask[:, 40:r1, 64:] = torch.rand(B, r1 - 40, max(0, T - 64), generator=g) < 0.5
    if mask is not None:
        mask[..., T - 1] = False
        mask = mask.to(gpu)
    return rows, kc, vc, do, mask


def _run(case, mask_kind, gpu, dtype, scores, nsplit=0):
    from xdot.ops import flash

    B, R, N, Rc, H, D = case
    T = N * Rc
    rows, kc, vc, do, mask = _inputs(case, mask_kind, gpu, dtype)
    scale = 1.0 / math.sqrt(D)
    mk = flash.prepare_mask(mask, B, R, T)
    kb, vb = flash.gathered_to_btc(kc), flash.gathered_to_btc(vc)
    sb = None
    if scores:
        sb = torch.full((flash.score_buffer_numel(B, H, R, T),), float("nan"), device=gpu)
    out, lse = flash.fwd(rows, kb, vb, mk, H, scale, nsplit=nsplit, fp32_mode=0, sbuf=sb)
    dkv, delta = flash.bwd_cols(do, rows, kb, vb, out, lse, mk, H, scale, fp32_mode=0, sbuf=sb)
    drows = flash.bwd_rows(do, rows, kb, vb, lse, delta, mk, H, scale, nsplit=nsplit, fp32_mode=0, sbuf=sb)
    C = H * D
    return (rows, kc, vc, do, mask), (out, lse, drows, dkv[..., :C], dkv[..., C:])


def _check(case, inputs, got, tol):
    B, R, N, Rc, H, D = case
    rows, kc, vc, do, mask = inputs
    out, lse, drows, dkc, dvc = got
    k, q, v, ref_o, ref_lse = _ref64(rows.float(), kc.float(), vc.float(), mask, H, 1.0 / math.sqrt(D))
    assert _rel(out, ref_o) <= tol, f"fwd out {_rel(out, ref_o):.2e}"
    assert (lse.double() - ref_lse).abs().max().item() < 50 * tol
    ref_o.backward(do.double())
    dkc, dvc = _to_gathered_btc(dkc, N), _to_gathered_btc(dvc, N)
    for what, g_, ref in (("d rows", drows, k.grad.transpose(1, 2).reshape(B, R, H * D)),
                          ("d cols (q)", dkc, _to_gathered(q.grad, N, B, Rc, H * D)),
                          ("d cols (v)", dvc, _to_gathered(v.grad, N, B, Rc, H * D))):
        assert _rel(g_, ref) <= tol, f"{what}: {_rel(g_, ref):.2e}"


def _to_gathered_btc(x, N):
    from xdot.ops import flash

    return flash.btc_to_rank_major(x.contiguous(), N)


@pytest.mark.parametrize("case", WIDE_CASES)
@pytest.mark.parametrize("mask_kind", ["none", "random", "blocks"])
def test_flash_wide_bf16(gpu, case, mask_kind):
    inputs, got = _run(case, mask_kind, gpu, torch.bfloat16, scores=False)
    for t in got:
        assert torch.isfinite(t).all()
    _check(case, inputs, got, 2e-2)


@pytest.mark.parametrize("case", WIDE_CASES)
@pytest.mark.parametrize("mask_kind", ["none", "random", "blocks"])
def test_flash_wide_f32(gpu, case, mask_kind):
    D = case[-1]
    modes = [True] if D > 256 else [True, False]
    res = []
    for scores in modes:
        inputs, got = _run(case, mask_kind, gpu, torch.float32, scores=scores)
        _check(case, inputs, got, 2e-6)
        res.append(got)
    if len(res) == 2:  # the score buffer changes nothing (same MFMA chains)
        for a, b in zip(*res):
            assert torch.equal(a, b)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_flash_wide_column_split(gpu, dtype):
    case = (1, 150, 1, 1000, 2, 256)
    _, ref = _run(case, "blocks", gpu, dtype, scores=dtype == torch.float32, nsplit=1)
    _, got = _run(case, "blocks", gpu, dtype, scores=dtype == torch.float32, nsplit=4)
    tol = 1e-6 if dtype == torch.float32 else 1e-2
    for a, b in zip(ref, got):
        assert _rel(b, a) <= tol


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("cfg", [(768, 2, 600), (256, 1, 500)])
def test_module_reference_configs_flash(gpu, dtype, cfg):
    """The reference's example.py (768 features, 2 heads) and test_gradient.py (256 features, one
    head) configurations run the fused flash path (no materialised scores) and match the fp64
    dense module: output, input gradient and every parameter gradient."""
    import xdot
    from xdot.utils.comm import LocalComm, use_comm

    dim, heads, T = cfg
    torch.manual_seed(0)
    with use_comm(LocalComm()):
        m = xdot.DistributedDotProductAttn(dim, num_heads=heads, add_bias=True).to(gpu, dtype)
        x = torch.randn(1, T, dim, device=gpu).to(dtype).requires_grad_(True)
        assert m._pick_impl(x) == "flash"
        ref = xdot.DistributedDotProductAttn(dim, num_heads=heads, add_bias=True, distributed=False,
                                             impl="materialized", backend="torch").to(gpu, torch.float64)
        ref.load_state_dict({k: v.double() for k, v in m.state_dict().items()})
        mask = torch.rand(1, T, T, device=gpu) < 0.3
        mask[..., 0] = False
        out = m(x, x, x, mask)
        out.float().square().sum().backward()
        xd = x.detach().double().requires_grad_(True)
        ro = ref(xd, xd, xd, mask)
        ro.square().sum().backward()
    tol = 1e-5 if dtype == torch.float32 else 2e-2
    assert _rel(out, ro) <= tol
    assert _rel(x.grad, xd.grad) <= 10 * tol
    rg = {n: q.grad for n, q in ref.named_parameters()}
    for n, p in m.named_parameters():
        if n == "queries.bias":  # zero in exact arithmetic (softmax shift invariance)
            continue
        assert _rel(p.grad, rg[n]) <= 10 * tol, n


def test_flash_wide_long_context_h2(gpu):
    """T = 200000, d = 768, h = 2 (D = 384) forward + backward at N = 1 in bf16 — the reference
    example's head shape at the long-context length (a materialised path would need 160 GB of bf16
    scores per head).  Sampled rows / columns recomputed in fp32."""
    import time

    from xdot.ops import flash

    R = T = 200_000
    H, D = 2, 384
    C = H * D
    scale = 1.0 / math.sqrt(D)
    g = torch.Generator(device=gpu).manual_seed(11)
    rows = torch.randn(1, R, C, device=gpu, generator=g).to(torch.bfloat16)
    qv = torch.randn(1, T, 2 * C, device=gpu, generator=g).to(torch.bfloat16)
    do = torch.randn(1, R, C, device=gpu, generator=g).to(torch.bfloat16)
    kc, vc = qv[..., :C], qv[..., C:]
    rk = flash.prescale(rows, scale)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out, lse = flash.fwd(rk, kc, vc, None, H, scale, prescaled=True)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    delta, lse2 = flash.bwd_prep(do, out, lse, H)
    dkv, _ = flash.bwd_cols(do, rk, kc, vc, out, lse, None, H, scale, delta, prescaled=True, lse2=lse2)
    drows = flash.bwd_rows(do, rk, kc, vc, lse, delta, None, H, scale, prescaled=True)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"\nT=200000 h=2 D=384 bf16: fwd {1e3 * (t1 - t0):.1f} ms, bwd {1e3 * (t2 - t1):.1f} ms")
    for h in range(H):
        sl = slice(h * D, (h + 1) * D)
        Q, K, V, dO = rows[0, :, sl].float(), kc[0, :, sl].float(), vc[0, :, sl].float(), do[0, :, sl].float()
        ri = torch.randint(0, R, (16,), device=gpu, generator=g)
        s = (Q[ri] @ K.t()) * scale
        lse_ref = torch.logsumexp(s, -1)
        p = torch.exp(s - lse_ref[:, None])
        o_ref = p @ V
        assert _rel(out[0, ri, sl], o_ref) <= 2e-2
        d_ref = (dO[ri] * out[0, ri, sl].float()).sum(-1)
        ds = p * ((dO[ri] @ V.t()) - d_ref[:, None])
        assert _rel(drows[0, ri, sl], scale * (ds @ K)) <= 3e-2
        cj = torch.randint(0, T, (16,), device=gpu, generator=g)
        sc = (Q @ K[cj].t()) * scale
        pc = torch.exp(sc - lse[0, h][:, None])
        dsc = pc * ((dO @ V[cj].t()) - delta[0, h][:, None])
        assert _rel(dkv[0, cj, C + h * D:C + (h + 1) * D], pc.t() @ dO) <= 3e-2
        assert _rel(dkv[0, cj, sl], scale * (dsc.t() @ Q)) <= 3e-2


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("cfg", [dict(key_dim=320, num_heads=4), dict(key_dim=64, value_dim=128, num_heads=1),
                                 dict(key_dim=384, value_dim=192, num_heads=1)])
def test_module_padded_heads_flash(gpu, dtype, cfg):
    """Head dims no kernel takes (80), or a value width different from the key width (num_heads =
    1, the reference's only such case: module.py:28-38) run the flash path on zero-padded heads
    (flash_head_dim) and match the fp64 dense module."""
    import xdot
    from xdot.parallel.attention import flash_head_dim
    from xdot.utils.comm import LocalComm, use_comm

    T = 400
    torch.manual_seed(1)
    with use_comm(LocalComm()):
        m = xdot.DistributedDotProductAttn(**cfg).to(gpu, dtype)
        dk, dv = m.dim, m.value_dim // m.num_heads
        assert flash_head_dim(dk, dv) not in (None, dk) or dk != dv
        xk = torch.randn(1, T, cfg["key_dim"], device=gpu).to(dtype).requires_grad_(True)
        xv = torch.randn(1, T, cfg.get("value_dim", cfg["key_dim"]), device=gpu).to(dtype).requires_grad_(True)
        assert m._pick_impl(xk) == "flash"
        ref = xdot.DistributedDotProductAttn(**cfg, distributed=False, impl="materialized",
                                             backend="torch").to(gpu, torch.float64)
        ref.load_state_dict({k: v.double() for k, v in m.state_dict().items()})
        out = m(xk, xk, xv, None)
        out.float().square().sum().backward()
        xkd = xk.detach().double().requires_grad_(True)
        xvd = xv.detach().double().requires_grad_(True)
        ro = ref(xkd, xkd, xvd, None)
        ro.square().sum().backward()
    tol = 1e-5 if dtype == torch.float32 else 2e-2
    assert _rel(out, ro) <= tol
    assert _rel(xk.grad, xkd.grad) <= 10 * tol and _rel(xv.grad, xvd.grad) <= 10 * tol
    for (n, p), (_, q) in zip(m.named_parameters(), ref.named_parameters()):
        assert _rel(p.grad, q.grad) <= 10 * tol, n


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_flash_wide_row_splits(gpu, monkeypatch, dtype):
    """Split counts of the wide kernels from their own occupancy (XDOT_WIDE_SPLIT): row splits of
    both column passes (fp32 partials, ordered sum into the output dtype) and column splits of the
    forward / row side; forced 2 / 3 and the automatic choice against the unsplit run and fp64."""
    case = (1, 2100, 1, 1500, 2, 256)  # 66 row tiles, 47 column tiles
    monkeypatch.setenv("XDOT_WIDE_SPLIT", "0")
    inputs, base = _run(case, "blocks", gpu, dtype, scores=dtype == torch.float32, nsplit=0)
    tol = 1e-6 if dtype == torch.float32 else 1e-2
    for sp in ("2", "3", "auto"):
        monkeypatch.setenv("XDOT_WIDE_SPLIT", sp)
        _, got = _run(case, "blocks", gpu, dtype, scores=dtype == torch.float32, nsplit=0)
        for a, b in zip(base, got):
            assert torch.isfinite(b).all()
            assert _rel(b, a) <= tol, f"splits {sp}: {_rel(b, a):.2e}"
        _check(case, inputs, got, 2e-6 if dtype == torch.float32 else 2e-2)


def _fp32_wide_module(gpu):
    import xdot

    torch.manual_seed(3)
    m = xdot.DistributedDotProductAttn(768, num_heads=2, impl="flash", distributed=False).to(gpu)
    x = torch.randn(1, 160, 768, device=gpu)
    mask = torch.rand(1, 160, 160, device=gpu) < 0.3
    mask[..., -1] = False
    return m, x, mask


def test_fp32_wide_retain_graph_twice(gpu):
    """Exact fp32 D = 384 (the reference example's heads), backward twice through a retained graph:
    with the separate dS buffer (default) S is intact, so the second pass gives the same gradients
    again (the first backward used to drop the buffer and the second failed)."""
    m, x, mask = _fp32_wide_module(gpu)
    loss = m(x, x, x, mask).square().mean()
    loss.backward(retain_graph=True)
    g1 = [p.grad.clone() for p in m.parameters()]
    loss.backward()
    for p, a in zip(m.parameters(), g1):
        torch.testing.assert_close(p.grad, 2 * a, rtol=1e-5, atol=1e-9)


def test_fp32_wide_retain_graph_in_place_raises(gpu, monkeypatch):
    """In the in-place score-buffer mode (no dS buffer) the first backward overwrites S; a second
    backward at fp32 D = 384 (no recompute kernel) must fail with a clear error, not a launch code."""
    from xdot.utils.env import FLAGS

    monkeypatch.setattr(FLAGS, "fp32_scores_dsbuf", False)
    m, x, mask = _fp32_wide_module(gpu)
    loss = m(x, x, x, mask).square().mean()
    loss.backward(retain_graph=True)
    with pytest.raises(RuntimeError, match="retained graph"):
        loss.backward()


def test_fp32_no_grad_forward_takes_no_score_buffer(gpu, monkeypatch):
    """no_grad / inference forwards never allocate the fp32 score buffers, and the
    wide exact-fp32 forward then runs the non-storing kernel (same output as with the buffer)."""
    from xdot.ops import flash

    calls = []
    orig = flash.score_buffers
    monkeypatch.setattr(flash, "score_buffers", lambda *a, **k: calls.append(a) or orig(*a, **k))
    m, x, mask = _fp32_wide_module(gpu)
    with torch.no_grad():
        y0 = m(x, x, x, mask)
    assert calls == []
    y1 = m(x, x, x, mask)
    assert len(calls) == 1
    torch.testing.assert_close(y0, y1.detach(), rtol=1e-6, atol=1e-7)
