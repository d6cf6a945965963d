"""fp32 flash kernels vs an fp64 PyTorch reference (GPU only): the exact family
(csrc/flash_f32.hip, fp32_mode=0: relative Frobenius error <= 2e-6, measured 3e-7..6e-7) and
the opt-in split-bf16 family (csrc/flash_x3.hip, fp32_mode=1: <= 2e-5, measured 6e-6..9e-6).

The reference module runs in fp32 (module.py:60-71); bf16 kernels would be at ~1e-2.  Head dims 32-128, ragged R / T, rank-
major gathered layouts, masks with fully masked tiles, column splits, a fully masked row
(NaN parity), the module's default fp32 path, and T = 200000 at the N=8 per-rank shape.
"""
import math

import pytest
import torch

from test_flash_gpu import CASES, _to_gathered

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return ((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30)).item()


def _ref64(rows, kc, vc, mask, H, scale):
    N, B, Rc, C = kc.shape
    R, D, T = rows.shape[1], C // H, N * Rc
    k = rows.double().view(B, R, H, D).transpose(1, 2).clone().requires_grad_(True)
    q = kc.double().permute(1, 0, 2, 3).reshape(B, T, H, D).transpose(1, 2).clone().requires_grad_(True)
    v = vc.double().permute(1, 0, 2, 3).reshape(B, T, H, D).transpose(1, 2).clone().requires_grad_(True)
    s = (k @ q.transpose(-1, -2)) * scale
    if mask is not None:
        s = s.masked_fill(mask.unsqueeze(1), -float("inf"))
    lse = torch.logsumexp(s, -1)
    o = torch.softmax(s, -1) @ v
    return k, q, v, o.transpose(1, 2).reshape(B, R, C), lse


def _inputs(case, mask_kind, gpu):
    B, R, N, Rc, H, D = case
    C, T = H * D, N * Rc
    g = torch.Generator(device="cpu").manual_seed(sum(case) + 1)
    rows = torch.randn(B, R, C, generator=g).to(gpu)
    kc = torch.randn(N, B, Rc, C, generator=g).to(gpu)
    vc = torch.randn(N, B, Rc, C, generator=g).to(gpu)
    do = torch.randn(B, R, C, generator=g).to(gpu)
    mask = None
    if mask_kind == "random":
        mask = torch.rand(B, R, T, generator=g) < 0.4
    elif mask_kind == "blocks":
        mask = torch.zeros(B, R, T, dtype=torch.bool)
        mask[:, :, : min(T, 128)] = True
        r1 = min(R, 90)
        mask[:, 40:r1, 128:] = torch.rand(B, r1 - 40, max(0, T - 128), generator=g) < 0.5
    if mask is not None:
        mask[..., T - 1] = False
        mask = mask.to(gpu)
    return rows, kc, vc, do, mask


@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("mask_kind", ["none", "random", "blocks"])
def test_flash_f32_fwd_bwd(gpu, case, mask_kind):
    from xdot.ops import flash

    B, R, N, Rc, H, D = case
    T = N * Rc
    rows, kc, vc, do, mask = _inputs(case, mask_kind, gpu)
    scale = 1.0 / math.sqrt(D)
    mk = flash.prepare_mask(mask, B, R, T)
    kb, vb = flash.gathered_to_btc(kc), flash.gathered_to_btc(vc)
    out, lse = flash.fwd(rows, kb, vb, mk, H, scale, fp32_mode=0)
    assert out.dtype == torch.float32
    k, q, v, ref_o, ref_lse = _ref64(rows, kc, vc, mask, H, scale)
    assert _rel(out, ref_o) <= 2e-6, f"fwd out {_rel(out, ref_o):.2e}"
    assert (lse.double() - ref_lse).abs().max().item() < 1e-5
    drows, dkc, dvc = flash.bwd(do, rows, kb, vb, out, lse, mk, H, scale, fp32_mode=0)
    dkc, dvc = flash.btc_to_rank_major(dkc, N), flash.btc_to_rank_major(dvc, N)
    ref_o.backward(do.double())
    for what, got, ref in (("d rows", drows, k.grad.transpose(1, 2).reshape(B, R, H * D)),
                           ("d cols (q)", dkc, _to_gathered(q.grad, N, B, Rc, H * D)),
                           ("d cols (v)", dvc, _to_gathered(v.grad, N, B, Rc, H * D))):
        assert got.dtype == torch.float32
        assert _rel(got, ref) <= 2e-6, f"{what}: {_rel(got, ref):.2e}"


@pytest.mark.parametrize("nsplit", [2, 5])
def test_flash_f32_column_split(gpu, nsplit):
    from xdot.ops import flash

    case = (1, 150, 1, 1000, 2, 96)
    rows, kc, vc, do, mask = _inputs(case, "blocks", gpu)
    kb, vb = flash.gathered_to_btc(kc), flash.gathered_to_btc(vc)
    mk = flash.prepare_mask(mask, 1, 150, 1000)
    o1, l1 = flash.fwd(rows, kb, vb, mk, 2, 0.1, nsplit=1, fp32_mode=0)
    o2, l2 = flash.fwd(rows, kb, vb, mk, 2, 0.1, nsplit=nsplit, fp32_mode=0)
    assert _rel(o2, o1) <= 1e-6 and (l1 - l2).abs().max().item() < 1e-5
    dkv, delta = flash.bwd_cols(do, rows, kb, vb, o1, l1, mk, 2, 0.1, fp32_mode=0)
    d1 = flash.bwd_rows(do, rows, kb, vb, l1, delta, mk, 2, 0.1, nsplit=1, fp32_mode=0)
    d2 = flash.bwd_rows(do, rows, kb, vb, l1, delta, mk, 2, 0.1, nsplit=nsplit, fp32_mode=0)
    assert _rel(d2, d1) <= 1e-6


# ---- exact fp32, score-buffer mode (XDOT_FP32_SCORES: S stored by the forward, dS by the column
# kernel; csrc/flash_f32.hip) -------------------------------------------------------------------
@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("mask_kind", ["none", "random", "blocks"])
@pytest.mark.parametrize("nsplit", [0, 3])
@pytest.mark.parametrize("direct,passes", [(False, 3), (True, 3), (True, 4)])
def test_flash_f32_score_buffer_bitwise(gpu, monkeypatch, case, mask_kind, nsplit, direct, passes):
    """Reading S / dS from the score buffer instead of recomputing them changes nothing: the
    forward, both backward kernels and the column-split partials are BITWISE equal to the
    recompute path (same MFMA chains), which the fp64 test above bounds.  ``direct``: the forward
    scatters S straight to the buffer (XDOT_F32_FWD_DIRECT=1, three workgroups per CU); ``passes``
    4: the fused column pass (dP, dQ and dV in one kernel, S -> dS in place)."""
    from xdot.ops import flash

    monkeypatch.setenv("XDOT_F32_FWD_DIRECT", "1" if direct else "0")

    B, R, N, Rc, H, D = case
    T = N * Rc
    rows, kc, vc, do, mask = _inputs(case, mask_kind, gpu)
    scale = 1.0 / math.sqrt(D)
    mk = flash.prepare_mask(mask, B, R, T)
    kb, vb = flash.gathered_to_btc(kc), flash.gathered_to_btc(vc)
    o1, l1 = flash.fwd(rows, kb, vb, mk, H, scale, nsplit=nsplit, fp32_mode=0)
    dkv1, dl1 = flash.bwd_cols(do, rows, kb, vb, o1, l1, mk, H, scale, fp32_mode=0)
    dr1 = flash.bwd_rows(do, rows, kb, vb, l1, dl1, mk, H, scale, nsplit=nsplit, fp32_mode=0)
    sb = torch.full((flash.score_buffer_numel(B, H, R, T),), float("nan"), device=gpu)  # no stale zeros
    o2, l2 = flash.fwd(rows, kb, vb, mk, H, scale, nsplit=nsplit, fp32_mode=0, sbuf=sb)
    dkv2, dl2 = flash.bwd_cols(do, rows, kb, vb, o2, l2, mk, H, scale, fp32_mode=0, sbuf=sb, passes=passes)
    dr2 = flash.bwd_rows(do, rows, kb, vb, l2, dl2, mk, H, scale, nsplit=nsplit, fp32_mode=0, sbuf=sb)
    assert torch.equal(o1, o2) and torch.equal(l1, l2)
    assert torch.equal(dkv1, dkv2), f"d cols {_rel(dkv2, dkv1):.2e}"
    assert torch.equal(dr1, dr2), f"d rows {_rel(dr2, dr1):.2e}"


def test_flash_f32_score_buffer_checks(gpu):
    """Wrong-sized buffers and non-fp32 inputs are refused on the host."""
    from xdot.ops import flash

    rows = torch.randn(1, 64, 128, device=gpu)
    kc = torch.randn(1, 96, 128, device=gpu)
    n = flash.score_buffer_numel(1, 2, 64, 96)
    assert n == (2 * 2 * 3 + 1) * 1024  # + the dump block
    for fm in (0, 1):
        with pytest.raises(RuntimeError, match="score buffer"):
            flash.fwd(rows, kc, kc, None, 2, 0.1, fp32_mode=fm, sbuf=torch.empty(n - 1, device=gpu))
    with pytest.raises(RuntimeError, match="fp32"):
        flash.fwd(rows.bfloat16(), kc.bfloat16(), kc.bfloat16(), None, 2, 0.1, sbuf=torch.empty(n, device=gpu))


def test_module_fp32_fused_cols(gpu, monkeypatch):
    """XDOT_F32_FUSED_COLS=1 (one fused column pass, one in-place score buffer) at a shape with
    column row splits: loss and gradients within 1e-6 of the two-pass default, fp64-bounded like
    the rest, and deterministic run to run."""
    import xdot
    from xdot.utils.comm import LocalComm, use_comm
    from xdot.utils.env import FLAGS

    def run(fused):
        monkeypatch.setattr(FLAGS, "f32_fused_cols", fused)
        torch.manual_seed(0)
        with use_comm(LocalComm()):
            m = xdot.DistributedDotProductAttn(384, num_heads=4, add_bias=True).to(gpu)
            x = torch.randn(1, 2600, 384, device=gpu, requires_grad=True)
            mask = torch.rand(1, 2600, 2600, device=gpu) < 0.2
            mask[..., 0] = False
            loss = m(x, x, x, mask).square().mean()
            loss.backward()
        return loss.detach(), [p.grad.clone() for p in m.parameters()] + [x.grad.clone()]

    la, a = run(False)
    lb, b = run(True)
    lc, c = run(True)
    assert torch.equal(lb, lc) and all(torch.equal(u, v) for u, v in zip(b, c))
    assert _rel(lb, la) <= 1e-6
    for u, v in zip(a, b):
        assert _rel(v, u) <= 1e-6


def test_module_fp32_score_buffer_matches_recompute(gpu):
    """The fp32 module with the score buffer (default) and without (XDOT_FP32_SCORES=0) gives
    bitwise equal outputs and gradients, twice in a row (determinism), and a retained graph's
    second backward (the buffer then holds dS: the recompute path runs) gives the same again."""
    import xdot
    from xdot.utils.comm import LocalComm, use_comm
    from xdot.utils.env import FLAGS

    def run(scores):
        old = FLAGS.fp32_scores
        FLAGS.fp32_scores = scores
        try:
            torch.manual_seed(0)
            with use_comm(LocalComm()):
                m = xdot.DistributedDotProductAttn(256, num_heads=4, add_bias=True).to(gpu)
                x = torch.randn(1, 700, 256, device=gpu, requires_grad=True)
                mask = torch.rand(1, 700, 700, device=gpu) < 0.2
                mask[..., 0] = False
                loss = m(x, x, x, mask).square().sum()
                loss.backward(retain_graph=True)
                g1 = [p.grad.clone() for p in m.parameters()] + [x.grad.clone()]
                loss.backward()
                g2 = [p.grad.clone() for p in m.parameters()] + [x.grad.clone()]
            return loss.detach(), g1, g2
        finally:
            FLAGS.fp32_scores = old

    la, a1, a2 = run(True)
    lb, b1, b2 = run(False)
    lc, c1, c2 = run(True)
    assert torch.equal(la, lb) and torch.equal(la, lc)
    for x, y, z in zip(a1, b1, c1):
        assert torch.equal(x, y) and torch.equal(x, z)
    for x, y in zip(a2, b2):
        assert torch.equal(x, y)


@pytest.mark.parametrize("fm", [0, 1])
def test_flash_f32_fully_masked_row_nan(gpu, fm):
    from xdot.ops import flash

    rows = torch.randn(1, 64, 128, device=gpu)
    kc = torch.randn(1, 96, 128, device=gpu)
    mask = torch.zeros(1, 64, 96, dtype=torch.bool, device=gpu)
    mask[0, 5] = True
    out, _ = flash.fwd(rows, kc, kc, flash.prepare_mask(mask, 1, 64, 96), 2, 0.125, fp32_mode=fm)
    assert torch.isnan(out[0, 5]).all() and not torch.isnan(out[0, 4]).any()


def test_module_fp32_default_is_fused(gpu):
    """An fp32 module takes the fused path by default (no (B,H,R,T) scores; exact fp32 kernels)
    and matches the fp64 dense module: outputs, input grads and all eight parameter grads."""
    import xdot
    from xdot.utils.comm import LocalComm, use_comm

    torch.manual_seed(0)
    D, H, T = 384, 4, 500
    with use_comm(LocalComm()):
        m = xdot.DistributedDotProductAttn(D, num_heads=H, add_bias=True).to(gpu)
        x = torch.randn(1, T, D, device=gpu, requires_grad=True)
        assert m._pick_impl(x) == "flash"
        ref = xdot.DistributedDotProductAttn(D, num_heads=H, add_bias=True, distributed=False,
                                             impl="materialized", backend="torch").to(gpu, torch.float64)
        ref.load_state_dict({k: v.double() for k, v in m.state_dict().items()})
        mask = torch.rand(1, T, T, device=gpu) < 0.3
        mask[..., 0] = False
        out = m(x, x, x, mask)
        out.square().sum().backward()
        xd = x.detach().double().requires_grad_(True)
        ro = ref(xd, xd, xd, mask)
        ro.square().sum().backward()
    assert _rel(out, ro) <= 1e-5
    assert _rel(x.grad, xd.grad) <= 1e-4
    rg = {n: q.grad for n, q in ref.named_parameters()}
    for n, p in m.named_parameters():
        if n == "queries.bias":  # exactly zero in exact arithmetic (softmax shift invariance)
            assert (p.grad.double() - rg[n]).norm().item() <= 1e-4 * rg["keys.bias"].norm().item()
            continue
        assert _rel(p.grad, rg[n]) <= 1e-4, n


@pytest.mark.parametrize("fm", [0, 1])
def test_flash_f32_long_context_sampled(gpu, fm):
    """T = 200000 in fp32 at the N=8 per-rank shape (R = 25000), both fp32 kernel families: no
    score tensor exists (a materialised fp32 (R, T) block alone would be 20 GB per head);
    sampled rows/columns are recomputed exactly in fp64."""
    from xdot.ops import flash

    R, T, H, D = 25_000, 200_000, 1, 96
    scale = 1.0 / math.sqrt(D)
    g = torch.Generator(device=gpu).manual_seed(7)
    rows = torch.randn(1, R, D, device=gpu, generator=g)
    kc = torch.randn(1, T, D, device=gpu, generator=g)
    vc = torch.randn(1, T, D, device=gpu, generator=g)
    do = torch.randn(1, R, D, device=gpu, generator=g)
    out, lse = flash.fwd(rows, kc, vc, None, H, scale, fp32_mode=fm)
    dkv, delta = flash.bwd_cols(do, rows, kc, vc, out, lse, None, H, scale, fp32_mode=fm)
    drows = flash.bwd_rows(do, rows, kc, vc, lse, delta, None, H, scale, fp32_mode=fm)
    K, V, Q, dO = kc[0].double(), vc[0].double(), rows[0].double(), do[0].double()
    ri = torch.randint(0, R, (16,), device=gpu, generator=g)
    s = (Q[ri] @ K.t()) * scale
    lse_ref = torch.logsumexp(s, -1)
    p = torch.exp(s - lse_ref[:, None])
    o_ref = p @ V
    assert _rel(out[0, ri], o_ref) <= 2e-5
    d_ref = (dO[ri] * o_ref).sum(-1)
    ds = p * ((dO[ri] @ V.t()) - d_ref[:, None])
    assert _rel(drows[0, ri], scale * (ds @ K)) <= 5e-5
    cj = torch.randint(0, T, (16,), device=gpu, generator=g)
    sc = (Q @ K[cj].t()) * scale
    pc = torch.exp(sc - lse[0, 0].double()[:, None])
    dsc = pc * ((dO @ V[cj].t()) - delta[0, 0].double()[:, None])
    assert _rel(dkv[0, cj, D:], pc.t() @ dO) <= 5e-5
    assert _rel(dkv[0, cj, :D], scale * (dsc.t() @ Q)) <= 5e-5


# ---- split-bf16 fp32 mode (csrc/flash_x3.hip, XDOT_FP32_MODE=split, opt-in) ---------------------
SPLIT_TOL = 2e-5  # measured 6e-6..9e-6 on every case (profiles/r3_fp32_split.md)


@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("mask_kind", ["none", "random", "blocks"])
def test_flash_split_fwd_bwd(gpu, case, mask_kind):
    """fp32 inputs on the bf16 matrix pipe (hi/lo split, 3 products): fp32 outputs within the
    split mode's bound of the fp64 reference, NaN-free, and closer than a plain bf16 pass."""
    from xdot.ops import flash

    B, R, N, Rc, H, D = case
    T = N * Rc
    rows, kc, vc, do, mask = _inputs(case, mask_kind, gpu)
    scale = 1.0 / math.sqrt(D)
    mk = flash.prepare_mask(mask, B, R, T)
    kb, vb = flash.gathered_to_btc(kc), flash.gathered_to_btc(vc)
    out, lse = flash.fwd(rows, kb, vb, mk, H, scale, fp32_mode=1)
    assert out.dtype == torch.float32
    k, q, v, ref_o, ref_lse = _ref64(rows, kc, vc, mask, H, scale)
    assert _rel(out, ref_o) <= SPLIT_TOL, f"fwd out {_rel(out, ref_o):.2e}"
    assert (lse.double() - ref_lse).abs().max().item() < 1e-4
    drows, dkc, dvc = flash.bwd(do, rows, kb, vb, out, lse, mk, H, scale, fp32_mode=1)
    dkc, dvc = flash.btc_to_rank_major(dkc, N), flash.btc_to_rank_major(dvc, N)
    ref_o.backward(do.double())
    for what, got, ref in (("d rows", drows, k.grad.transpose(1, 2).reshape(B, R, H * D)),
                           ("d cols (q)", dkc, _to_gathered(q.grad, N, B, Rc, H * D)),
                           ("d cols (v)", dvc, _to_gathered(v.grad, N, B, Rc, H * D))):
        assert got.dtype == torch.float32
        assert _rel(got, ref) <= SPLIT_TOL, f"{what}: {_rel(got, ref):.2e}"


@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("mask_kind", ["none", "random", "blocks"])
@pytest.mark.parametrize("nsplit", [0, 3])
def test_flash_split_score_buffer(gpu, case, mask_kind, nsplit):
    """Split mode with the score buffer (forward stores S, dV pass + dQ pass read it and write
    dS, the row kernel reads dS): within the split bound of the fp64 reference.  Not bitwise
    equal to the recompute path: its column kernel recomputes S with the operand roles of the
    3-term split swapped (another rounding order); the buffer carries the forward's own S."""
    from xdot.ops import flash

    B, R, N, Rc, H, D = case
    T = N * Rc
    rows, kc, vc, do, mask = _inputs(case, mask_kind, gpu)
    scale = 1.0 / math.sqrt(D)
    mk = flash.prepare_mask(mask, B, R, T)
    kb, vb = flash.gathered_to_btc(kc), flash.gathered_to_btc(vc)
    sb = torch.full((flash.score_buffer_numel(B, H, R, T),), float("nan"), device=gpu)  # no stale zeros
    out, lse = flash.fwd(rows, kb, vb, mk, H, scale, nsplit=nsplit, fp32_mode=1, sbuf=sb)
    o1, l1 = flash.fwd(rows, kb, vb, mk, H, scale, nsplit=nsplit, fp32_mode=1)
    assert torch.equal(out, o1) and torch.equal(lse, l1)  # storing S changes nothing
    k, q, v, ref_o, ref_lse = _ref64(rows, kc, vc, mask, H, scale)
    dkv, delta = flash.bwd_cols(do, rows, kb, vb, out, lse, mk, H, scale, fp32_mode=1, sbuf=sb)
    drows = flash.bwd_rows(do, rows, kb, vb, lse, delta, mk, H, scale, nsplit=nsplit, fp32_mode=1, sbuf=sb)
    C = H * D
    dkc, dvc = flash.btc_to_rank_major(dkv[..., :C], N), flash.btc_to_rank_major(dkv[..., C:], N)
    ref_o.backward(do.double())
    for what, got, ref in (("d rows", drows, k.grad.transpose(1, 2).reshape(B, R, H * D)),
                           ("d cols (q)", dkc, _to_gathered(q.grad, N, B, Rc, H * D)),
                           ("d cols (v)", dvc, _to_gathered(v.grad, N, B, Rc, H * D))):
        assert torch.isfinite(got).all(), what
        assert _rel(got, ref) <= SPLIT_TOL, f"{what}: {_rel(got, ref):.2e}"


def test_flash_split_column_split_and_exact_module(gpu):
    """Split mode through the column-split partial path; the fused module under
    XDOT_FP32_MODE=split (opt-in split-bf16 kernels) at the split family's bound."""
    import xdot
    from xdot.ops import flash
    from xdot.utils.comm import LocalComm, use_comm
    from xdot.utils.env import FLAGS

    case = (1, 150, 1, 1000, 2, 96)
    rows, kc, vc, do, mask = _inputs(case, "blocks", gpu)
    kb, vb = flash.gathered_to_btc(kc), flash.gathered_to_btc(vc)
    mk = flash.prepare_mask(mask, 1, 150, 1000)
    o1, l1 = flash.fwd(rows, kb, vb, mk, 2, 0.1, nsplit=1, fp32_mode=1)
    o2, l2 = flash.fwd(rows, kb, vb, mk, 2, 0.1, nsplit=3, fp32_mode=1)
    # split partials sum the ~1e-5 product errors in another order than one pass
    assert _rel(o2, o1) <= 2e-5 and (l1 - l2).abs().max().item() < 1e-5
    dkv, delta = flash.bwd_cols(do, rows, kb, vb, o1, l1, mk, 2, 0.1, fp32_mode=1)
    d1 = flash.bwd_rows(do, rows, kb, vb, l1, delta, mk, 2, 0.1, nsplit=1, fp32_mode=1)
    d2 = flash.bwd_rows(do, rows, kb, vb, l1, delta, mk, 2, 0.1, nsplit=4, fp32_mode=1)
    assert _rel(d2, d1) <= 2e-5

    torch.manual_seed(0)
    D, H, T = 384, 4, 500
    old = FLAGS.fp32_mode
    try:
        with use_comm(LocalComm()):
            m = xdot.DistributedDotProductAttn(D, num_heads=H, add_bias=True).to(gpu)
            x = torch.randn(1, T, D, device=gpu, requires_grad=True)
            ref = xdot.DistributedDotProductAttn(D, num_heads=H, add_bias=True, distributed=False,
                                                 impl="materialized", backend="torch").to(gpu, torch.float64)
            ref.load_state_dict({k: v.double() for k, v in m.state_dict().items()})
            FLAGS.fp32_mode = "split"
            out = m(x, x, x, None)
            out.square().sum().backward()
            xd = x.detach().double().requires_grad_(True)
            ro = ref(xd, xd, xd, None)
            ro.square().sum().backward()
    finally:
        FLAGS.fp32_mode = old
    assert _rel(out, ro) <= 3e-5
    assert _rel(x.grad, xd.grad) <= 1e-4


# ---- column-side row splits (BwdArgs::csq / csv, XDOT_CSPLIT): the fp32 column kernels cut the
# R rows into s ranges against the last-round tail; fp32 partials are summed in order ------------
@pytest.mark.parametrize("fm", [0, 1])
@pytest.mark.parametrize("mode", ["recompute", "inplace", "dsbuf"])
def test_flash_f32_column_row_splits(gpu, monkeypatch, fm, mode):
    """Row splits 2 / 3 / 4 and the automatic choice match the unsplit column grads (another
    summation order: <= 1e-6 exact, <= 2e-5 split family) and the fp64 reference; the dQ-first
    + separate-dS schedule runs each pass with its own split count."""
    from xdot.ops import flash

    case = (1, 2100, 1, 1500, 2, 96)  # 66 row tiles: up to 4 splits of >= 16
    B, R, N, Rc, H, D = case
    T, C = N * Rc, H * D
    rows, kc, vc, do, mask = _inputs(case, "blocks", gpu)
    scale = 1.0 / math.sqrt(D)
    mk = flash.prepare_mask(mask, B, R, T)
    kb, vb = flash.gathered_to_btc(kc), flash.gathered_to_btc(vc)
    tol = 1e-6 if fm == 0 else 2e-5

    def cols():
        if mode == "recompute":
            o, l = flash.fwd(rows, kb, vb, mk, H, scale, fp32_mode=fm)
            return flash.bwd_cols(do, rows, kb, vb, o, l, mk, H, scale, fp32_mode=fm)[0]
        sb = torch.full((flash.score_buffer_numel(B, H, R, T),), float("nan"), device=gpu)
        o, l = flash.fwd(rows, kb, vb, mk, H, scale, fp32_mode=fm, sbuf=sb)
        if mode == "inplace":
            return flash.bwd_cols(do, rows, kb, vb, o, l, mk, H, scale, fp32_mode=fm, sbuf=sb)[0]
        ds = torch.full_like(sb, float("nan"))
        dkv, dl = flash.bwd_cols(do, rows, kb, vb, o, l, mk, H, scale, fp32_mode=fm, sbuf=sb, dsbuf=ds, passes=2)
        flash.bwd_cols(do, rows, kb, vb, o, l, mk, H, scale, delta=dl, fp32_mode=fm, sbuf=sb, dsbuf=ds,
                       passes=1, out_dkv=dkv)
        return dkv

    monkeypatch.setenv("XDOT_CSPLIT", "1")
    base = cols()
    k, q, v, ref_o, _ = _ref64(rows, kc, vc, mask, H, scale)
    ref_o.backward(do.double())
    refq, refv = _to_gathered(q.grad, N, B, Rc, C), _to_gathered(v.grad, N, B, Rc, C)
    for s in ("2", "3", "4", "auto"):
        monkeypatch.setenv("XDOT_CSPLIT", s)
        got = cols()
        assert torch.isfinite(got).all(), s
        assert _rel(got, base) <= tol, f"splits {s}: {_rel(got, base):.2e}"
        for what, g_, r_ in (("q", got[..., :C], refq), ("v", got[..., C:], refv)):
            err = _rel(flash.btc_to_rank_major(g_.contiguous(), N), r_)
            assert err <= (2e-6 if fm == 0 else 2e-5), f"splits {s} d cols ({what}): {err:.2e}"


# ---- dS-only buffer mode (XDOT_FP32_DS_ONLY): the forward stores nothing, the single-pass column
# kernel recomputes S and stores dS, the row kernel reads it --------------------------------------
@pytest.mark.parametrize("fm", [0, 1])
@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("mask_kind", ["none", "blocks"])
def test_flash_f32_ds_only_buffer(gpu, fm, case, mask_kind):
    """Column grads are bitwise those of the recompute path (same kernel, plus a store); the row
    grad from the stored dS is bitwise that of the S + dS buffer mode in the exact family (same
    dS chain), and within each family's fp64 bound either way."""
    from xdot.ops import flash

    B, R, N, Rc, H, D = case
    T = N * Rc
    rows, kc, vc, do, mask = _inputs(case, mask_kind, gpu)
    scale = 1.0 / math.sqrt(D)
    mk = flash.prepare_mask(mask, B, R, T)
    kb, vb = flash.gathered_to_btc(kc), flash.gathered_to_btc(vc)
    out, lse = flash.fwd(rows, kb, vb, mk, H, scale, fp32_mode=fm)
    dkv1, dl1 = flash.bwd_cols(do, rows, kb, vb, out, lse, mk, H, scale, fp32_mode=fm)
    ds = torch.full((flash.score_buffer_numel(B, H, R, T),), float("nan"), device=gpu)
    dkv2, dl2 = flash.bwd_cols(do, rows, kb, vb, out, lse, mk, H, scale, fp32_mode=fm, dsbuf=ds)
    assert torch.equal(dkv1, dkv2) and torch.equal(dl1, dl2)
    drows = flash.bwd_rows(do, rows, kb, vb, lse, dl2, mk, H, scale, fp32_mode=fm, dsbuf=ds)
    k, q, v, ref_o, _ = _ref64(rows, kc, vc, mask, H, scale)
    ref_o.backward(do.double())
    ref = k.grad.transpose(1, 2).reshape(B, R, H * D)
    assert torch.isfinite(drows).all()
    assert _rel(drows, ref) <= (2e-6 if fm == 0 else SPLIT_TOL), f"d rows {_rel(drows, ref):.2e}"
    if fm == 0:
        sb = torch.full_like(ds, float("nan"))
        o3, l3 = flash.fwd(rows, kb, vb, mk, H, scale, fp32_mode=0, sbuf=sb)
        _, dl3 = flash.bwd_cols(do, rows, kb, vb, o3, l3, mk, H, scale, fp32_mode=0, sbuf=sb)
        d3 = flash.bwd_rows(do, rows, kb, vb, l3, dl3, mk, H, scale, fp32_mode=0, sbuf=sb)
        assert torch.equal(d3, drows)


@pytest.mark.parametrize("mode", ["all", "none"])
def test_module_fp32_ds_only_mode(gpu, monkeypatch, mode):
    """The module's fp32 paths under XDOT_FP32_DS_ONLY=all / none against fp64 torch."""
    import xdot
    from xdot.utils.comm import LocalComm, use_comm
    from xdot.utils.env import FLAGS

    torch.manual_seed(0)
    Dm, H, T = 384, 4, 700
    old = (FLAGS.fp32_ds_only, FLAGS.fp32_mode)
    try:
        with use_comm(LocalComm()):
            m = xdot.DistributedDotProductAttn(Dm, num_heads=H, add_bias=True).to(gpu)
            ref = xdot.DistributedDotProductAttn(Dm, num_heads=H, add_bias=True, distributed=False,
                                                 impl="materialized", backend="torch").to(gpu, torch.float64)
            ref.load_state_dict({k: v.double() for k, v in m.state_dict().items()})
            xd = torch.randn(1, T, Dm, device=gpu, dtype=torch.float64)
            mask = torch.rand(1, T, T, device=gpu) < 0.2
            mask[..., 0] = False
            xr = xd.clone().requires_grad_(True)
            ro = ref(xr, xr, xr, mask)
            ro.square().sum().backward()
            FLAGS.fp32_ds_only = mode
            for fmode, tol in (("exact", 1e-5), ("split", 3e-5)):  # as the module tests above
                FLAGS.fp32_mode = fmode
                x = xd.float().requires_grad_(True)
                out = m(x, x, x, mask)
                out.square().sum().backward()
                assert _rel(out, ro) <= tol, (fmode, _rel(out, ro))
                assert _rel(x.grad, xr.grad) <= 1e-4, (fmode, _rel(x.grad, xr.grad))
                m.zero_grad()
    finally:
        FLAGS.fp32_ds_only, FLAGS.fp32_mode = old


@pytest.mark.parametrize("mask_kind", ["none", "random"])
def test_flash_f32_head_heavy_forward(gpu, mask_kind):
    """Exact-fp32 forward on the head-heavy grid (R = 97 row blocks x 8 heads = 776 blocks: each
    XCD's 96 resident slots run its first 96 blocks whole, its last block in column pieces merged
    by the tail combine): vs fp64 (<= 2e-6) and vs a forced uniform column split (<= 1e-6); a
    fully masked row inside a tail block gives NaN output and -inf LSE like the reference."""
    from xdot.ops import flash

    B, R, H, D, T = 1, 97 * 128, 8, 96, 1024
    C = H * D
    g = torch.Generator(device="cpu").manual_seed(11)
    rows = torch.randn(B, R, C, generator=g).to(gpu)
    kc = torch.randn(1, B, T, C, generator=g).to(gpu)
    vc = torch.randn(1, B, T, C, generator=g).to(gpu)
    mask = None
    if mask_kind == "random":
        mask = torch.rand(B, R, T, generator=g) < 0.1
        mask[..., 0] = False
        mask[:, R - 16, :] = True  # a fully masked row in the last (tail) row block of every head
        mask = mask.to(gpu)
    scale = 1.0 / math.sqrt(D)
    mk = flash.prepare_mask(mask, B, R, T)
    kb, vb = flash.gathered_to_btc(kc), flash.gathered_to_btc(vc)
    sb = torch.full((flash.score_buffer_numel(B, H, R, T),), float("nan"), device=gpu)
    o, lse = flash.fwd(rows, kb, vb, mk, H, scale, fp32_mode=0, sbuf=sb)
    ou, lu = flash.fwd(rows, kb, vb, mk, H, scale, nsplit=2, fp32_mode=0)
    _, _, _, o64, l64 = _ref64(rows, kc, vc, mask, H, scale)
    ok = torch.ones(R, dtype=torch.bool, device=gpu)
    if mask is not None:
        ok[R - 16] = False
        assert torch.isnan(o[:, R - 16]).all() and torch.isneginf(lse[:, :, R - 16]).all()
        assert torch.isnan(ou[:, R - 16]).all()
    assert _rel(o[:, ok], o64[:, ok]) <= 2e-6
    assert _rel(lse[:, :, ok], l64[:, :, ok]) <= 2e-6
    assert _rel(o[:, ok], ou[:, ok]) <= 1e-6


@pytest.mark.parametrize("mask_kind", ["none", "random"])
def test_flash_f32_fused_cols_head_heavy(gpu, mask_kind):
    """The fused exact-fp32 column pass on its head-heavy grid (T = 65 column blocks x 8 heads =
    520 blocks: each XCD's 64 resident slots sweep 64 blocks whole, its last block in row pieces
    whose compact partials the tail sum adds) == the two-pass score-buffer path (uniform splits)
    to fp32 summation order, and the row side that reads its dS likewise."""
    from xdot.ops import flash

    B, R, H, D, T = 1, 2048, 8, 96, 65 * 128
    C = H * D
    g = torch.Generator(device="cpu").manual_seed(13)
    rows = torch.randn(B, R, C, generator=g).to(gpu)
    kc = torch.randn(1, B, T, C, generator=g).to(gpu)
    vc = torch.randn(1, B, T, C, generator=g).to(gpu)
    do = torch.randn(B, R, C, generator=g).to(gpu)
    mask = None
    if mask_kind == "random":
        mask = torch.rand(B, R, T, generator=g) < 0.1
        mask[..., 0] = False
        mask = mask.to(gpu)
    scale = 1.0 / math.sqrt(D)
    mk = flash.prepare_mask(mask, B, R, T)
    kb, vb = flash.gathered_to_btc(kc), flash.gathered_to_btc(vc)
    res = []
    for passes in (4, 3):
        sb = torch.full((flash.score_buffer_numel(B, H, R, T),), float("nan"), device=gpu)
        o, l = flash.fwd(rows, kb, vb, mk, H, scale, fp32_mode=0, sbuf=sb)
        dkv, dl = flash.bwd_cols(do, rows, kb, vb, o, l, mk, H, scale, fp32_mode=0, sbuf=sb, passes=passes)
        dr = flash.bwd_rows(do, rows, kb, vb, l, dl, mk, H, scale, fp32_mode=0, sbuf=sb)
        res.append((dkv, dr))
    (a1, r1), (a0, r0) = res
    assert torch.isfinite(a1).all()
    assert _rel(a1, a0) <= 1e-6, f"cols {_rel(a1, a0):.2e}"
    assert _rel(r1, r0) <= 1e-6, f"rows {_rel(r1, r0):.2e}"
