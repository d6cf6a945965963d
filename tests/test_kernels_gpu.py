"""Numerics of the gfx950 HIP kernels against plain fp32 PyTorch references (GPU only)."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

DTYPES = [torch.bfloat16, torch.float16, torch.float32]


def _tol(dt, k):
    if dt == torch.float32:
        return 1e-4 * math.sqrt(k)
    return (2e-2 if dt == torch.bfloat16 else 4e-3) * math.sqrt(max(k, 1) / 64)


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("a_mc,b_mc", [(False, False), (False, True), (True, False), (True, True)])
@pytest.mark.parametrize("M,N,K", [(128, 128, 32), (200, 77, 96), (513, 300, 130), (64, 1000, 8)])
def test_strided_gemm_layouts(gpu, dt, a_mc, b_mc, M, N, K):
    from xdot.ops.gemm import strided_gemm

    g = torch.Generator(device="cpu").manual_seed(M * 7 + N + K)
    A = torch.randn(2, M, K, generator=g) if not a_mc else torch.randn(2, K, M, generator=g)
    B = torch.randn(2, N, K, generator=g) if not b_mc else torch.randn(2, K, N, generator=g)
    Ad, Bd = A.to(gpu, dt), B.to(gpu, dt)
    C = torch.empty(2, M, N, device=gpu, dtype=torch.float32)
    strided_gemm(Ad, Bd, C, M=M, N=N, K=K, nb2=2, lda=(M if a_mc else K), ldb=(N if b_mc else K),
                 ldc=N, sA2=M * K, sB2=N * K, sC2=M * N, a_mc=a_mc, b_mc=b_mc, alpha=0.5)
    Af = Ad.float()
    Bf = Bd.float()
    opA = Af.transpose(-1, -2) if a_mc else Af
    opB = Bf if b_mc else Bf.transpose(-1, -2)
    ref = 0.5 * torch.matmul(opA, opB)
    err = (C - ref).abs().max().item()
    assert err <= _tol(dt, K) * max(1.0, ref.abs().max().item() / 4), err


@pytest.mark.parametrize("dt", DTYPES)
def test_gemm_segments_and_bf16_out(gpu, dt):
    """K segments (the fused sum over ranks of distributed_matmul_all)."""
    from xdot.ops.gemm import all_chunk_into

    N, Pn, R, c = 3, 2, 50, 40
    left = torch.randn(Pn, R, N * R, device=gpu).to(dt)
    chunk = torch.randn(N, Pn, R, c, device=gpu).to(dt)
    out = torch.zeros(Pn, R, c, device=gpu, dtype=dt)
    all_chunk_into(out, left, chunk, 0)
    ref = sum(left.float()[..., j * R:(j + 1) * R] @ chunk.float()[j] for j in range(N))
    assert torch.allclose(out.float(), ref, atol=_tol(dt, N * R) * 4, rtol=2e-2)


def test_gemm_integer_exact_fp32(gpu):
    """Exact small-integer products must be bit-exact in fp32 (reference tests use ==)."""
    from xdot.ops.gemm import matmul

    a = torch.randint(-8, 8, (3, 67, 45), device=gpu).float()
    b = torch.randint(-8, 8, (3, 45, 91), device=gpu).float()
    assert torch.equal(matmul(a, b), a @ b)


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("T", [8, 100, 2048, 25000, 70000])
def test_softmax_fwd_bwd(gpu, dt, T):
    from xdot.ops.softmax import scale_mask_softmax_fwd, scale_mask_softmax_bwd

    B, H, R = 1, 2, 3
    x = (torch.randn(B, H, R, T, device=gpu) * 3).to(dt)
    mask = torch.rand(B, R, T, device=gpu) < 0.3
    mask[..., 0] = False
    scale = 0.37
    y = scale_mask_softmax_fwd(x, mask, scale)
    ref = torch.softmax((x.float() * scale).masked_fill(mask.unsqueeze(1), -float("inf")), -1)
    atol = 1e-6 if dt == torch.float32 else 8e-3
    assert torch.allclose(y.float(), ref, atol=atol, rtol=2e-2)
    dy = torch.randn_like(x)
    dx = scale_mask_softmax_bwd(y, dy, scale)
    yf = y.float()
    dref = scale * yf * (dy.float() - (dy.float() * yf).sum(-1, keepdim=True))
    assert torch.allclose(dx.float(), dref, atol=atol * 4, rtol=3e-2)


def test_softmax_fully_masked_row_is_nan(gpu):
    from xdot.ops.softmax import scale_mask_softmax_fwd

    x = torch.randn(1, 1, 2, 64, device=gpu)
    mask = torch.zeros(1, 2, 64, dtype=torch.bool, device=gpu)
    mask[0, 1] = True
    y = scale_mask_softmax_fwd(x, mask, 1.0)
    assert torch.isnan(y[0, 0, 1]).all() and not torch.isnan(y[0, 0, 0]).any()


@pytest.mark.parametrize("K,M,N", [(25000, 768, 1536), (3125, 768, 768), (300, 96, 200), (7, 64, 64)])
def test_weight_grad_split_k(gpu, K, M, N):
    """split-K dW = dyᵀ·x (bf16 in, fp32 accumulation) vs an fp32 torch reference."""
    from xdot.ops.linear import weight_grad

    g = torch.Generator(device="cpu").manual_seed(K)
    dy = torch.randn(K, M, generator=g).to(gpu, torch.bfloat16)
    x = torch.randn(K, N, generator=g).to(gpu, torch.bfloat16)
    ref = dy.float().t() @ x.float()
    got = weight_grad(dy, x, torch.float32)
    torch.testing.assert_close(got, ref, rtol=1e-4, atol=1e-3 * ref.abs().max().item() ** 0.5)


def test_linear_fn_grads(gpu):
    from xdot.ops.linear import linear

    g = torch.Generator(device="cpu").manual_seed(3)
    x = torch.randn(2, 500, 96, generator=g).to(gpu, torch.bfloat16).requires_grad_(True)
    w = (0.1 * torch.randn(64, 96, generator=g)).to(gpu, torch.bfloat16).requires_grad_(True)
    b = torch.randn(64, generator=g).to(gpu, torch.bfloat16).requires_grad_(True)
    dy = torch.randn(2, 500, 64, generator=g).to(gpu, torch.bfloat16)
    y = linear(x, w, b)
    y.backward(dy)
    xr, wr, br = (t.detach().float().requires_grad_(True) for t in (x, w, b))
    torch.nn.functional.linear(xr, wr, br).backward(dy.float())
    torch.testing.assert_close(y.float(), torch.nn.functional.linear(xr, wr, br), rtol=2e-2, atol=5e-2)
    for a, r in ((x.grad, xr.grad), (w.grad, wr.grad), (b.grad, br.grad)):
        torch.testing.assert_close(a.float(), r, rtol=2e-2, atol=2e-2 * r.abs().max().item())


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_fused_adamw_kernel(gpu, dtype):
    """One multi-tensor HIP launch == torch.optim.AdamW on fp32 copies (fp32 moments)."""
    from xdot.ops.optim import FusedAdamW

    g = torch.Generator(device="cpu").manual_seed(5)
    shapes = [(768, 768), (1536, 768), (3,), (1000, 7)]
    p32 = [torch.randn(*s, generator=g) for s in shapes]
    gr = [torch.randn(*s, generator=g) for s in shapes]
    kw = dict(lr=3e-3, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.05)
    ours = [p.to(gpu, dtype).requires_grad_(True) for p in p32]
    # the last one starts one element into its storage: the kernel's unaligned (scalar) path
    buf = torch.zeros(1 + p32[3].numel(), device=gpu, dtype=dtype)
    buf[1:].copy_(p32[3].flatten().to(gpu, dtype))
    ours[3] = buf[1:].view(p32[3].shape).detach().requires_grad_(True)
    ref = [p.to(gpu).requires_grad_(True) for p in p32]
    o1, o2 = FusedAdamW(ours, **kw), torch.optim.AdamW(ref, **kw)
    for s in range(3):
        for p, q, x in zip(ours, ref, gr):
            p.grad = (x * (s + 1)).to(gpu, dtype)
            q.grad = p.grad.float()
        o1.step()
        o2.step()
    for p, q in zip(ours, ref):
        tol = 1e-6 if dtype == torch.float32 else 2e-2
        torch.testing.assert_close(p.float(), q.detach(), rtol=tol, atol=tol)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("offset", [24, 100, None])
def test_all_row_chunking_gpu(gpu, dt, offset):
    """distributed_matmul_all with an offset: row-block plan (fp32 K-accumulation through the
    GEMM's beta) and the reference's feature-column plan agree with torch (world size 1)."""
    import xdot.parallel.functional as F
    from xdot.utils.comm import LocalComm

    g = torch.Generator(device="cpu").manual_seed(7)
    left = torch.randn(2, 300, 300, generator=g).to(gpu, dt)
    right = torch.randn(2, 300, 256, generator=g).to(gpu, dt)
    ref = left.float() @ right.float()
    for chunking in ("rows", "columns"):
        out = F.distributed_matmul_all(left, right, offset, comm=LocalComm(), chunking=chunking)
        assert out.dtype == dt
        tol = 1e-3 if dt == torch.float32 else 0.15
        assert (out.float() - ref).abs().max().item() < tol * ref.abs().max().item() ** 0.5, chunking


def test_cast_multi_kernel(gpu):
    """csrc/optim.hip cast_multi (GradSync's 16-bit <-> fp32 conversions, one launch for many
    pairs) against torch's .to(): every dtype pair, sizes with and without a full 8-element tail,
    offset (not 16-byte aligned) views, more pairs than one launch holds."""
    import xdot._ext as ext

    g = torch.Generator(device="cpu").manual_seed(3)
    dts = [torch.float32, torch.bfloat16, torch.float16]
    srcs, dsts = [], []
    for i, n in enumerate([1, 7, 8, 9, 2048, 2049, 768 * 768, 40001] * 5):
        sdt, ddt = dts[i % 3], dts[(i // 3) % 3]
        base = (torch.randn(n + 3, generator=g) * 4).to(gpu, sdt)
        srcs.append(base[3:] if i % 4 == 1 else base[:n])  # offset views: scalar path
        out = torch.full((n + 1,), float("nan"), device=gpu, dtype=ddt)
        dsts.append(out[1:] if i % 5 == 2 else out[:n])
    assert len(srcs) > 32
    ext.ops().cast_multi(srcs, dsts)
    for s, d in zip(srcs, dsts):
        torch.testing.assert_close(d, s.to(d.dtype), rtol=0, atol=0)


def test_fused_adamw_fp32_grads(gpu):
    """FusedAdamW.step(params=, grads=) with fp32 gradients of bf16 parameters (GradSync's reduced
    sums): the update uses the fp32 values and writes each, rounded, into p.grad (one launch);
    == torch.optim.AdamW on fp32 copies; a parameter without an override uses its own p.grad."""
    from xdot.ops.optim import FusedAdamW

    g = torch.Generator(device="cpu").manual_seed(9)
    shapes = [(768, 768), (1536, 768), (5,), (999, 7)]
    p32 = [torch.randn(*s, generator=g) for s in shapes]
    gr = [torch.randn(*s, generator=g) for s in shapes]
    kw = dict(lr=3e-3, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.05)
    ours = [p.to(gpu, torch.bfloat16).requires_grad_(True) for p in p32]
    buf = torch.zeros(1 + p32[3].numel(), device=gpu, dtype=torch.bfloat16)  # unaligned: scalar path
    buf[1:].copy_(p32[3].flatten().to(gpu, torch.bfloat16))
    ours[3] = buf[1:].view(p32[3].shape).detach().requires_grad_(True)
    ref = [p.to(gpu).requires_grad_(True) for p in p32]
    o1, o2 = FusedAdamW(ours, **kw), torch.optim.AdamW(ref, **kw)
    for s in range(3):
        g32 = [(x * (s + 1)).to(gpu) for x in gr]
        for p, q, x in zip(ours, ref, g32):
            q.grad = x.clone()
            p.grad = None
        ours[2].grad = g32[2].to(torch.bfloat16)  # no override: its own bf16 gradient
        q2 = ref[2]
        q2.grad = ours[2].grad.float()
        o1.step(params=ours, grads=[g32[0], g32[1], None, g32[3]])
        o2.step()
        for i in (0, 1, 3):
            torch.testing.assert_close(ours[i].grad, g32[i].to(torch.bfloat16), rtol=0, atol=0)
    for p, q in zip(ours, ref):
        torch.testing.assert_close(p.float(), q.detach(), rtol=2e-2, atol=2e-2)
