"""Flash-attention kernels (csrc/flash_*.hip) vs an fp32 PyTorch reference (GPU only).

Covers every head dim, bf16/fp16, ragged R (not a multiple of 128) and T (not a multiple
of 64), batch > 1 with a rank-major gathered layout (N > 1 chunks), no mask / random mask /
structured mask with fully-masked tiles and a fully-masked row (NaN parity).
"""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu


def _ref(rows, kc, vc, mask, H, scale):
    """fp32 reference: returns out, lse, and a closure for grads."""
    N, B, Rc, C = kc.shape
    R = rows.shape[1]
    D = C // H
    T = N * Rc
    k = rows.float().view(B, R, H, D).transpose(1, 2).clone().requires_grad_(True)
    q = kc.float().permute(1, 0, 2, 3).reshape(B, T, H, D).transpose(1, 2).clone().requires_grad_(True)
    v = vc.float().permute(1, 0, 2, 3).reshape(B, T, H, D).transpose(1, 2).clone().requires_grad_(True)
    s = (k @ q.transpose(-1, -2)) * scale
    if mask is not None:
        s = s.masked_fill(mask.unsqueeze(1), -float("inf"))
    lse = torch.logsumexp(s, -1)
    p = torch.softmax(s, -1)
    o = p @ v
    return k, q, v, o.transpose(1, 2).reshape(B, R, C), lse


def _close(what, a, b, fro, elem=10.0):
    """rel. Frobenius error <= fro, and |a - b| <= elem * fro * (|b| + 0.25 rms(b)) everywhere."""
    a, b = a.float(), b.float()
    assert torch.isfinite(a).all(), f"{what}: non-finite"
    err = ((a - b).norm() / b.norm().clamp_min(1e-12)).item()
    assert err <= fro, f"{what}: relative Frobenius error {err:.3e} > {fro:.1e}"
    rms = b.pow(2).mean().sqrt()
    bound = elem * fro * (b.abs() + 0.25 * rms)
    worst = ((a - b).abs() / bound).max().item()
    assert worst <= 1.0, f"{what}: an element is {worst:.2f}x past its bound"


def _to_gathered(x, N, B, Rc, C):  # (B, H, T, D) grad -> (N, B, Rc, C)
    H, D = x.shape[1], x.shape[3]
    return x.transpose(1, 2).reshape(B, N, Rc, H * D).permute(1, 0, 2, 3)


CASES = [
    # (B, R, N, Rc, H, D)
    (1, 256, 1, 256, 2, 96),
    (1, 200, 1, 200, 4, 64),
    (2, 130, 3, 70, 2, 128),
    (1, 77, 2, 100, 3, 32),
    (1, 300, 4, 75, 8, 96),
]


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("mask_kind", ["none", "random", "blocks"])
@pytest.mark.parametrize("prescaled", [False, True])
def test_flash_fwd_bwd(gpu, dt, case, mask_kind, prescaled):
    """``prescaled``: the kernels read rows * scale * log2 e (flash.prescale, the module's
    default) and seed their score accumulators; gradients are still those of the unscaled rows."""
    from xdot.ops import flash

    B, R, N, Rc, H, D = case
    C, T = H * D, N * Rc
    g = torch.Generator(device="cpu").manual_seed(sum(case))
    rows = torch.randn(B, R, C, generator=g).to(gpu, dt)
    kc = torch.randn(N, B, Rc, C, generator=g).to(gpu, dt)
    vc = torch.randn(N, B, Rc, C, generator=g).to(gpu, dt)
    mask = None
    if mask_kind == "random":
        mask = torch.rand(B, R, T, generator=g) < 0.4
    elif mask_kind == "blocks":
        mask = torch.zeros(B, R, T, dtype=torch.bool)
        mask[:, :, : min(T, 128)] = True           # fully masked tiles
        r1 = min(R, 90)
        mask[:, 40:r1, 128:] = torch.rand(B, r1 - 40, max(0, T - 128), generator=g) < 0.5
    if mask is not None:
        mask[..., T - 1] = False                   # keep every row alive
        mask = mask.to(gpu)
    scale = 1.0 / math.sqrt(D)
    mk = flash.prepare_mask(mask, B, R, T)
    rk = flash.prescale(rows, scale) if prescaled else rows
    out, lse = flash.fwd(rk, flash.gathered_to_btc(kc), flash.gathered_to_btc(vc), mk, H, scale, prescaled=prescaled)
    k, q, v, ref_o, ref_lse = _ref(rows, kc, vc, mask, H, scale)
    # relative Frobenius error, and every element against a per-element bound (|b| plus a
    # small share of the tensor's RMS for entries near zero): tens-of-percent errors on any
    # part of the output fail
    fro = 1e-2 if dt == torch.bfloat16 else 3e-3
    _close("fwd out", out, ref_o, fro)
    assert (lse - ref_lse).abs().max().item() < 1e-2, "lse"

    do = torch.randn(B, R, C, generator=g).to(gpu, dt)
    drows, dkc, dvc = flash.bwd(do, rk, flash.gathered_to_btc(kc), flash.gathered_to_btc(vc), out, lse, mk, H, scale,
                                prescaled=prescaled)
    dkc, dvc = flash.btc_to_rank_major(dkc, N), flash.btc_to_rank_major(dvc, N)
    ref_o.backward(do.float())
    dk_ref = k.grad.transpose(1, 2).reshape(B, R, C)
    dq_ref = _to_gathered(q.grad, N, B, Rc, C)
    dv_ref = _to_gathered(v.grad, N, B, Rc, C)

    gfro = 1.5e-2 if dt == torch.bfloat16 else 4e-3
    _close("d rows", drows, dk_ref, gfro)
    _close("d cols (q)", dkc, dq_ref, gfro)
    _close("d cols (v)", dvc, dv_ref, gfro)


@pytest.mark.parametrize("prescaled", [False, True])
def test_flash_fully_masked_row_nan(gpu, prescaled):
    from xdot.ops import flash

    B, R, N, Rc, H, D = 1, 64, 1, 64, 2, 64
    rows = torch.randn(B, R, H * D, device=gpu, dtype=torch.bfloat16)
    kc = torch.randn(N, B, Rc, H * D, device=gpu, dtype=torch.bfloat16)
    mask = torch.zeros(B, R, N * Rc, dtype=torch.bool, device=gpu)
    mask[0, 5] = True
    kb = flash.gathered_to_btc(kc)
    rk = flash.prescale(rows, 0.125) if prescaled else rows
    out, lse = flash.fwd(rk, kb, kb, flash.prepare_mask(mask, B, R, N * Rc), H, 0.125, prescaled=prescaled)
    assert torch.isnan(out[0, 5]).all()
    assert not torch.isnan(out[0, 4]).any()


def test_mask_pack_flags(gpu):
    from xdot.ops import flash

    B, R, T = 2, 70, 150
    mask = torch.zeros(B, R, T, dtype=torch.bool, device=gpu)
    mask[0, :, :64] = True
    mask[1, 3, 100] = True
    mk = flash.prepare_mask(mask, B, R, T)
    assert mk.bits.shape == (B, 3, R) and mk.flags.shape == (B, 3, 4)
    f = mk.flags.cpu()[..., :3]
    assert f[0, :, 0].tolist() == [1, 1, 1] and f[0, :, 1:].eq(0).all()
    assert f[1, 0, 1] == 2 and f[1, 1:, :].eq(0).all()
    bits = mk.bits.cpu().view(torch.int64)
    assert bits[1, 1, 3].item() == (1 << (100 - 64))


@pytest.mark.parametrize("shape", [(2, 70, 150), (1, 200, 1000), (1, 64, 128), (1, 100, 300), (2, 70, 1501),
                                   (1, 130, 12500)])
def test_mask_pack_column_major(gpu, shape):
    """bits_t (B, ceil(R/64), Tpad): bit i of word (b, rt, t) == mask[b, 64*rt + i, t]; and the
    row-major bits (B, NKT, R).  Row strides 8-, 4- and 1-byte aligned (T = 1000 / 300 / 1501)."""
    from xdot.ops import flash

    B, R, T = shape
    g = torch.Generator(device="cpu").manual_seed(R)
    mask = torch.rand(B, R, T, generator=g) < 0.3
    mk = flash.prepare_mask(mask.to(gpu), B, R, T)
    NRT, Tpad = (R + 63) // 64, (T + 127) // 128 * 128
    assert mk.bits_t.shape == (B, NRT, Tpad)
    bt = mk.bits_t.cpu().view(torch.int64)
    ref = torch.zeros(B, NRT * 64, Tpad, dtype=torch.bool)
    ref[:, :R, :T] = mask
    ref = ref.view(B, NRT, 64, Tpad)
    got = torch.stack([(bt >> i) & 1 for i in range(64)], dim=2).bool()   # (B, NRT, 64, Tpad)
    assert torch.equal(got, ref)
    NKT = (T + 63) // 64
    bits = mk.bits.cpu().view(torch.int64)                                # (B, NKT, R)
    rowbits = torch.stack([(bits >> i) & 1 for i in range(64)], dim=-1).bool()  # (B, NKT, R, 64)
    refr = torch.zeros(B, R, NKT * 64, dtype=torch.bool)
    refr[..., :T] = mask
    assert torch.equal(rowbits.permute(0, 2, 1, 3).reshape(B, R, NKT * 64), refr)


@pytest.mark.parametrize("nsplit", [2, 5])
@pytest.mark.parametrize("masked", [False, True])
def test_flash_column_split(gpu, nsplit, masked):
    """Column-split forward (+ combine) and split row-side backward match the unsplit kernels."""
    from xdot.ops import flash

    B, R, T, H, D = 1, 150, 1000, 2, 96
    g = torch.Generator(device="cpu").manual_seed(nsplit)
    rows = torch.randn(B, R, H * D, generator=g).to(gpu, torch.bfloat16)
    kc = torch.randn(B, T, H * D, generator=g).to(gpu, torch.bfloat16)
    vc = torch.randn(B, T, H * D, generator=g).to(gpu, torch.bfloat16)
    mask = None
    if masked:
        mask = (torch.rand(B, R, T, generator=g) < 0.5)
        mask[:, :, :400] = True      # whole splits fully masked for every row
        mask[..., -1] = False
        mask = mask.to(gpu)
    mk = flash.prepare_mask(mask, B, R, T)
    o1, l1 = flash.fwd(rows, kc, vc, mk, H, 0.1, nsplit=1)
    o2, l2 = flash.fwd(rows, kc, vc, mk, H, 0.1, nsplit=nsplit)
    assert (o1.float() - o2.float()).abs().max().item() < 2e-2
    assert (l1 - l2).abs().max().item() < 1e-3
    do = torch.randn(B, R, H * D, generator=g).to(gpu, torch.bfloat16)
    dkv, delta = flash.bwd_cols(do, rows, kc, vc, o1, l1, mk, H, 0.1)
    d1 = flash.bwd_rows(do, rows, kc, vc, l1, delta, mk, H, 0.1, nsplit=1)
    d2 = flash.bwd_rows(do, rows, kc, vc, l1, delta, mk, H, 0.1, nsplit=nsplit)
    assert (d1.float() - d2.float()).abs().max().item() <= 2e-2 * d1.float().abs().max().item()


@pytest.mark.parametrize("D,dt", [(64, torch.bfloat16), (96, torch.bfloat16), (32, torch.float16), (128, torch.bfloat16)])
def test_flash_bwd_delta_and_given_delta(gpu, D, dt):
    """δ op == rowsum(dO·O) in fp32 (the 8-lanes-per-row prep kernel), lse2 == lse · log2 e;
    passing δ to bwd_cols gives the same gradients."""
    import math

    from xdot.ops import flash

    B, R, T, H = 2, 70, 300, 4
    g = torch.Generator(device="cpu").manual_seed(7)
    rows = torch.randn(B, R, H * D, generator=g).to(gpu, dt)
    kc = torch.randn(B, T, H * D, generator=g).to(gpu, dt)
    vc = torch.randn(B, T, H * D, generator=g).to(gpu, dt)
    do = torch.randn(B, R, H * D, generator=g).to(gpu, dt)
    o, lse = flash.fwd(rows, kc, vc, None, H, 0.125)
    delta = flash.bwd_delta(do, o, H)
    ref = (do.float() * o.float()).view(B, R, H, D).sum(-1).transpose(1, 2)
    torch.testing.assert_close(delta, ref, rtol=1e-4, atol=1e-4)
    delta2, lse2 = flash.bwd_prep(do, o, lse, H)
    assert torch.equal(delta2, delta)
    torch.testing.assert_close(lse2, lse * (1 / math.log(2)), rtol=1e-6, atol=1e-6)
    dkv1, d1 = flash.bwd_cols(do, rows, kc, vc, o, lse, None, H, 0.125)
    dkv2, d2 = flash.bwd_cols(do, rows, kc, vc, o, lse, None, H, 0.125, delta)
    assert d2.data_ptr() == delta.data_ptr()
    assert torch.equal(d1, delta) and torch.equal(dkv1, dkv2)


def test_flash_bwd_cols_input_dtype_output(gpu):
    """fp32_out=False rounds the same fp32 accumulators once to bf16: bitwise equal to
    casting the fp32 output."""
    from xdot.ops import flash

    B, R, T, H, D = 1, 130, 700, 2, 96
    g = torch.Generator(device="cpu").manual_seed(11)
    rows, kc, vc, do = (torch.randn(B, n, H * D, generator=g).to(gpu, torch.bfloat16) for n in (R, T, T, R))
    mask = (torch.rand(B, R, T, generator=g) < 0.3).to(gpu)
    mask[..., 0] = False
    mk = flash.prepare_mask(mask, B, R, T)
    o, lse = flash.fwd(rows, kc, vc, mk, H, 0.1)
    d32, _ = flash.bwd_cols(do, rows, kc, vc, o, lse, mk, H, 0.1)
    d16, _ = flash.bwd_cols(do, rows, kc, vc, o, lse, mk, H, 0.1, fp32_out=False)
    assert d32.dtype == torch.float32 and d16.dtype == torch.bfloat16
    assert torch.equal(d16, d32.to(torch.bfloat16))


def test_mask_cache_and_all_false_short_circuit(gpu):
    """The same mask tensor is packed once (flash.MASK_CACHE); an in-place write re-packs it;
    an all-False mask is handed out as None once its "anything masked?" copy has landed."""
    from xdot.ops import flash

    flash.MASK_CACHE.clear()
    B, R, T = 1, 64, 192  # 3 column tiles: the flag rows carry one padding tile
    z = torch.zeros(B, R, T, dtype=torch.bool, device=gpu)
    first = flash.prepare_mask_cached(z, B, R, T)
    assert first is not None and int(first.flags[..., :3].max()) == 0
    torch.cuda.synchronize()
    assert flash.prepare_mask_cached(z, B, R, T) is None
    m = torch.rand(B, R, T, device=gpu) < 0.3
    p1 = flash.prepare_mask_cached(m, B, R, T)
    torch.cuda.synchronize()
    p2 = flash.prepare_mask_cached(m, B, R, T)
    assert p2 is p1
    bits_before = p1.bits.clone()
    m[0, 0, :] = True  # in-place: _version bumps, the entry is stale
    p3 = flash.prepare_mask_cached(m, B, R, T)
    assert p3 is not p1 and not torch.equal(p3.bits, bits_before)
    torch.testing.assert_close(p3.bits, flash.prepare_mask(m, B, R, T).bits, atol=0, rtol=0)
    # a different tensor with the same contents is a different key (no stale hits by address)
    del m, p1, p2, p3
    m2 = torch.rand(B, R, T, device=gpu) < 0.5
    p4 = flash.prepare_mask_cached(m2, B, R, T)
    torch.testing.assert_close(p4.bits, flash.prepare_mask(m2, B, R, T).bits, atol=0, rtol=0)


def test_bf16_reduction_of_gathered_grads_bounded(gpu):
    """The fused path's default at N > 1: the gathered-side [dq | dv] partials are rounded once
    to bf16 in the kernel and RCCL's reduce-scatter sums them in bf16 (rounding after every
    add of its ring).  Emulate 8 ranks' partials and a bf16 ring sum, and pin the error
    against an fp64 reference: relative Frobenius <= 1.5e-2 (vs the fp32 reduction's)."""
    from xdot.ops import flash

    N, R, H, D = 8, 256, 2, 64
    C, T = H * D, N * R
    scale = 1.0 / math.sqrt(D)
    g = torch.Generator(device="cpu").manual_seed(11)
    kc = torch.randn(1, T, C, generator=g).to(gpu, torch.bfloat16)
    vc = torch.randn(1, T, C, generator=g).to(gpu, torch.bfloat16)
    rows = [torch.randn(1, R, C, generator=g).to(gpu, torch.bfloat16) for _ in range(N)]
    dos = [torch.randn(1, R, C, generator=g).to(gpu, torch.bfloat16) for _ in range(N)]
    p16, p32 = [], []
    for r in range(N):
        out, lse = flash.fwd(rows[r], kc, vc, None, H, scale)
        a, _ = flash.bwd_cols(dos[r], rows[r], kc, vc, out, lse, None, H, scale, fp32_out=False)
        b, _ = flash.bwd_cols(dos[r], rows[r], kc, vc, out, lse, None, H, scale, fp32_out=True)
        p16.append(a)
        p32.append(b)
    ring = p16[0].clone()
    for r in range(1, N):  # one rounding per ring step, as RCCL's bf16 reduce-scatter
        ring = (ring.float() + p16[r].float()).to(torch.bfloat16)
    red32 = sum(p.float() for p in p32)
    # fp64 reference of the summed gathered-side gradient
    k = torch.cat(rows, 1).double().view(1, T, H, D).transpose(1, 2)
    q = kc.double().view(1, T, H, D).transpose(1, 2).requires_grad_(True)
    v = vc.double().view(1, T, H, D).transpose(1, 2).requires_grad_(True)
    o = torch.softmax((k @ q.transpose(-1, -2)) * scale, -1) @ v
    o.backward(torch.cat(dos, 1).double().view(1, T, H, D).transpose(1, 2))
    ref = torch.cat([q.grad.transpose(1, 2).reshape(1, T, C), v.grad.transpose(1, 2).reshape(1, T, C)], -1)

    def rel(a):
        return ((a.double() - ref).norm() / ref.norm()).item()

    e16, e32 = rel(ring), rel(red32)
    print(f"bf16 ring reduction rel err {e16:.3e}, fp32 reduction {e32:.3e}")
    assert e32 <= 1e-2
    assert e16 <= 1.5e-2


@pytest.mark.parametrize("prescaled", [False, True])
def test_flash_head_heavy_grid(gpu, prescaled):
    """Whole-GPU forward with the head-heavy grid (bindings.cpp head_heavy_plan): each XCD runs
    its row blocks whole and splits only its last ones into column pieces (compact partials +
    flash_fwd_combine_tail).  R = 65 row blocks per head, 8 heads: 64 whole + 1 split tail block
    per XCD.  Checked against the fp32 reference, against the uniform nsplit = 1 launch, and a
    fully masked row inside a tail block must come out NaN."""
    from xdot.ops import flash

    B, R, T, H, D = 1, 65 * 128, 2048, 8, 64
    C = H * D
    g = torch.Generator(device="cpu").manual_seed(11)
    rows = torch.randn(B, R, C, generator=g).to(gpu, torch.bfloat16)
    kc = torch.randn(1, B, T, C, generator=g).to(gpu, torch.bfloat16)
    vc = torch.randn(1, B, T, C, generator=g).to(gpu, torch.bfloat16)
    mask = torch.rand(B, R, T, generator=g) < 0.3
    mask[:, :, :64] = True          # fully masked tiles
    mask[..., T - 1] = False
    mask[0, 64 * 128 + 9] = True    # a fully masked row in the split tail block
    mask = mask.to(gpu)
    scale = 1.0 / math.sqrt(D)
    mk = flash.prepare_mask(mask, B, R, T)
    rk = flash.prescale(rows, scale) if prescaled else rows
    kb, vb = flash.gathered_to_btc(kc), flash.gathered_to_btc(vc)
    out, lse = flash.fwd(rk, kb, vb, mk, H, scale, prescaled=prescaled)          # head-heavy (auto)
    o1, l1 = flash.fwd(rk, kb, vb, mk, H, scale, nsplit=1, prescaled=prescaled)  # uniform, whole blocks
    dead = 64 * 128 + 9
    assert torch.isnan(out[0, dead]).all() and torch.isnan(o1[0, dead]).all()
    keep = torch.ones(R, dtype=torch.bool, device=gpu)
    keep[dead] = False
    _, _, _, ref_o, ref_lse = _ref(rows, kc, vc, mask, H, scale)
    _close("fwd out", out[:, keep], ref_o[:, keep], 1e-2)
    assert (lse[..., keep] - ref_lse[..., keep]).abs().max().item() < 1e-2
    # whole blocks are bitwise the uniform launch's; tail rows agree to bf16 rounding
    assert torch.equal(out[:, : 64 * 128], o1[:, : 64 * 128])
    assert (out[:, keep].float() - o1[:, keep].float()).abs().max().item() < 2e-2


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("mask_kind", ["none", "blocks"])
def test_flash_cols_row_splits(gpu, monkeypatch, dt, mask_kind):
    """Row splits of the pipelined 16-bit column kernel (pre-scaled, D <= 96; BwdArgs::csq,
    XDOT_CSPLIT): fp32 partials of 2 / 3 / 4 row ranges and the automatic choice match the
    unsplit grads (fp32 output: <= 1e-5, another summation order of the same products; 16-bit
    output: one rounding) and the torch fp32 reference."""
    from xdot.ops import flash

    B, R, N, Rc, H, D = 1, 2600, 1, 1500, 2, 96  # 41 row tiles of 64
    C, T = H * D, N * Rc
    g = torch.Generator(device="cpu").manual_seed(7)
    rows = torch.randn(B, R, C, generator=g).to(gpu, dt)
    kc = torch.randn(N, B, Rc, C, generator=g).to(gpu, dt)
    vc = torch.randn(N, B, Rc, C, generator=g).to(gpu, dt)
    do = torch.randn(B, R, C, generator=g).to(gpu, dt)
    mask = None
    if mask_kind == "blocks":
        mask = torch.zeros(B, R, T, dtype=torch.bool)
        mask[:, :, :128] = True
        mask[:, 40:900, 128:] = torch.rand(B, 860, T - 128, generator=g) < 0.5
        mask[..., T - 1] = False
        mask = mask.to(gpu)
    scale = 1.0 / math.sqrt(D)
    mk = flash.prepare_mask(mask, B, R, T)
    rk = flash.prescale(rows, scale)
    kb, vb = flash.gathered_to_btc(kc), flash.gathered_to_btc(vc)
    out, lse = flash.fwd(rk, kb, vb, mk, H, scale, prescaled=True)

    def cols(fp32_out):
        return flash.bwd_cols(do, rk, kb, vb, out, lse, mk, H, scale, fp32_out=fp32_out, prescaled=True)[0]

    monkeypatch.setenv("XDOT_CSPLIT", "1")
    base32, base16 = cols(True), cols(False)
    k, q, v, ref_o, _ = _ref(rows, kc, vc, mask, H, scale)
    ref_o.backward(do.float())
    refq, refv = _to_gathered(q.grad, N, B, Rc, C), _to_gathered(v.grad, N, B, Rc, C)
    gfro = 1.5e-2 if dt == torch.bfloat16 else 4e-3
    for s in ("2", "3", "4", "auto"):
        monkeypatch.setenv("XDOT_CSPLIT", s)
        g32, g16 = cols(True), cols(False)
        assert g16.dtype == dt and g32.dtype == torch.float32
        r32 = ((g32 - base32).norm() / base32.norm()).item()
        r16 = ((g16.float() - base16.float()).norm() / base16.float().norm()).item()
        assert r32 <= 1e-5, f"splits {s}: fp32 out {r32:.2e}"
        assert r16 <= (8e-3 if dt == torch.bfloat16 else 1e-3), f"splits {s}: 16-bit out {r16:.2e}"
        _close(f"splits {s} d cols (q)", flash.btc_to_rank_major(g16[..., :C].contiguous(), N), refq, gfro)
        _close(f"splits {s} d cols (v)", flash.btc_to_rank_major(g16[..., C:].contiguous(), N), refv, gfro)
