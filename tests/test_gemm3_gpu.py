"""Numerics of the 8-phase 16x16x32 GEMM (csrc/gemm3.hip) against fp32 PyTorch (GPU only).

Every call forces the v3 path (``path=3`` raises if the kernel does not take the call): all four
operand layouts, edge tiles shifted inside the matrix, K tails (zero-filled DMA lanes), K
segments, split-K slices, fp32 and 16-bit outputs, persistent workgroups crossing items.
"""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

HALF = [torch.bfloat16, torch.float16]
LAYOUTS = [(False, False), (False, True), (True, False), (True, True)]


def _tol(dt, k):
    return (2e-2 if dt == torch.bfloat16 else 4e-3) * math.sqrt(max(k, 1) / 64)


def _run(gpu, dt, a_mc, b_mc, M, N, K, nseg=1, batches=2, alpha=1.0, out_dt=torch.float32, seed=0, path=3):
    from xdot.ops.gemm import strided_gemm

    g = torch.Generator(device="cpu").manual_seed(seed + M * 7 + N + K)
    A = torch.randn(batches, nseg, *((K, M) if a_mc else (M, K)), generator=g).to(gpu, dt)
    B = torch.randn(batches, nseg, *((K, N) if b_mc else (N, K)), generator=g).to(gpu, dt)
    C = torch.full((batches, M, N), float("nan"), device=gpu, dtype=out_dt)
    strided_gemm(A, B, C, M=M, N=N, K=K, nseg=nseg, nb2=batches, lda=(M if a_mc else K),
                 ldb=(N if b_mc else K), ldc=N, sA2=nseg * M * K, sB2=nseg * N * K, sC2=M * N,
                 sAseg=M * K, sBseg=N * K, a_mc=a_mc, b_mc=b_mc, alpha=alpha, path=path)
    Af, Bf = A.float(), B.float()
    opA = Af.transpose(-1, -2) if a_mc else Af        # (b, s, M, K)
    opB = Bf if b_mc else Bf.transpose(-1, -2)        # (b, s, K, N)
    ref = alpha * torch.matmul(opA, opB).sum(1)
    assert torch.isfinite(C.float()).all(), "unwritten output elements"
    err = (C.float() - ref).abs().max().item()
    tol = _tol(dt, K * nseg) * max(1.0, ref.abs().max().item() / 4)
    if out_dt != torch.float32:
        tol += ref.abs().max().item() * (2 ** -7 if out_dt == torch.bfloat16 else 2 ** -10)
    assert err <= tol, (err, tol)
    return C


@pytest.mark.parametrize("dt", HALF)
@pytest.mark.parametrize("a_mc,b_mc", LAYOUTS)
@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (520, 264, 96), (776, 1000, 40), (264, 520, 200), (256, 264, 8)])
def test_gemm3_layouts_tails(gpu, dt, a_mc, b_mc, M, N, K):
    _run(gpu, dt, a_mc, b_mc, M, N, K, alpha=0.5)


@pytest.mark.parametrize("a_mc,b_mc", LAYOUTS)
@pytest.mark.parametrize("out_dt", [torch.bfloat16, torch.float32])
def test_gemm3_segments(gpu, a_mc, b_mc, out_dt):
    """3 K segments with a K tail each: the k-tile stream crosses segment boundaries"""
    _run(gpu, torch.bfloat16, a_mc, b_mc, 512, 264, 104, nseg=3, alpha=0.25, out_dt=out_dt)


@pytest.mark.parametrize("a_mc,b_mc", [(False, False), (True, True), (False, True)])
@pytest.mark.parametrize("K", [4096, 4104])
def test_gemm3_split_k(gpu, a_mc, b_mc, K):
    """one 256x256 tile per batch and a long K: the dispatcher splits K (fp32 slices + reduce)"""
    _run(gpu, torch.bfloat16, a_mc, b_mc, 256, 256, K, batches=1, alpha=2.0, out_dt=torch.bfloat16)


@pytest.mark.parametrize("a_mc,b_mc", LAYOUTS)
def test_gemm3_persistent_many_items(gpu, a_mc, b_mc):
    """405 items on <= 256 workgroups: each persistent workgroup crosses item boundaries (shifted
    edge tiles, K tails, segments, batches) with the DMA stream running on"""
    _run(gpu, torch.bfloat16, a_mc, b_mc, 2056, 2056, 200, nseg=2, batches=5, alpha=0.5, out_dt=torch.bfloat16)


@pytest.mark.parametrize("K", [3125, 77, 1562, 12503])
@pytest.mark.parametrize("out_dt", [torch.bfloat16, torch.float32])
def test_gemm3_odd_k_both_mn_contiguous(gpu, K, out_dt):
    """K % 8 != 0 with both operands mn-contiguous (the weight gradients dYᵀ·X at T/N = 3125 rows):
    the K tail is zero-filled per k row, so gemm3 takes these shapes; split-K included."""
    _run(gpu, torch.bfloat16, True, True, 768, 768, K, batches=1, out_dt=out_dt)
    _run(gpu, torch.bfloat16, True, True, 1536, 768, K, batches=1, out_dt=out_dt, alpha=0.5)


def test_weight_grad_odd_rows(gpu):
    """xdot.ops.linear.weight_grad at the N=8 rank shape (K = 3125 rows) against fp32 torch."""
    from xdot.ops.linear import weight_grad

    g = torch.Generator(device="cpu").manual_seed(9)
    dy = torch.randn(3125, 1536, generator=g).to(gpu, torch.bfloat16)
    x = torch.randn(3125, 768, generator=g).to(gpu, torch.bfloat16)
    w = weight_grad(dy, x)
    ref = dy.float().t() @ x.float()
    assert ((w.float() - ref).norm() / ref.norm()).item() < 1e-2


def test_gemm3_odd_n_kc(gpu):
    """k-contiguous B with N % 8 != 0 (nt's per-rank column count at T/N = 3125): the last
    column tile is shifted by a non-multiple of 8 and stored through unaligned 16-byte stores"""
    _run(gpu, torch.bfloat16, False, False, 600, 3125, 96, batches=1, out_dt=torch.bfloat16)


def test_gemm3_matches_v2_bitwise_order(gpu):
    """same products as the v2 kernel within rounding (independent implementations)"""
    c3 = _run(gpu, torch.bfloat16, False, True, 1024, 768, 1000, batches=1, out_dt=torch.float32, path=3)
    c2 = _run(gpu, torch.bfloat16, False, True, 1024, 768, 1000, batches=1, out_dt=torch.float32, path=2)
    assert (c3 - c2).abs().max().item() < 1e-2


def test_gemm3_rejects_beta(gpu):
    from xdot.ops.gemm import strided_gemm

    A = torch.randn(256, 64, device=gpu, dtype=torch.bfloat16)
    C = torch.zeros(256, 256, device=gpu, dtype=torch.bfloat16)
    with pytest.raises(RuntimeError):
        strided_gemm(A, A, C, M=256, N=256, K=64, lda=64, ldb=64, ldc=256, beta=1.0, path=3)


def _rel_fro(x, ref):
    return ((x.double() - ref).norm() / ref.norm()).item()


@pytest.mark.parametrize("a_mc,b_mc", LAYOUTS)
@pytest.mark.parametrize("M,N,K,nseg", [(520, 776, 200, 1), (264, 296, 96, 3)])
def test_gemm3_split_fp32(gpu, a_mc, b_mc, M, N, K, nseg):
    """fp32 operands as hi/lo bf16 halves, three products on the bf16 pipe (path 4), against an
    fp64 reference: relative Frobenius error <= 2e-5 (exact fp32 is ~1e-7; bf16 ~3e-3)"""
    from xdot.ops.gemm import strided_gemm

    g = torch.Generator(device="cpu").manual_seed(M + N + K)
    batches = 2
    A = torch.randn(batches, nseg, *((K, M) if a_mc else (M, K)), generator=g, dtype=torch.float64)
    B = torch.randn(batches, nseg, *((K, N) if b_mc else (N, K)), generator=g, dtype=torch.float64)
    C = torch.full((batches, M, N), float("nan"), device=gpu)
    strided_gemm(A.float().to(gpu), B.float().to(gpu), C, M=M, N=N, K=K, nseg=nseg, nb2=batches,
                 lda=(M if a_mc else K), ldb=(N if b_mc else K), ldc=N, sA2=nseg * M * K, sB2=nseg * N * K,
                 sC2=M * N, sAseg=M * K, sBseg=N * K, a_mc=a_mc, b_mc=b_mc, alpha=0.5, path=4)
    Af, Bf = A.float().double(), B.float().double()   # the fp32 inputs, exactly
    opA = Af.transpose(-1, -2) if a_mc else Af
    opB = Bf if b_mc else Bf.transpose(-1, -2)
    ref = 0.5 * torch.matmul(opA, opB).sum(1)
    err = _rel_fro(C.cpu(), ref)
    assert err <= 2e-5, err


def test_gemm3_split_fp32_split_k(gpu):
    """split fp32 with split-K slices (one tile, long K)"""
    from xdot.ops.gemm import strided_gemm

    g = torch.Generator(device="cpu").manual_seed(5)
    A = torch.randn(256, 4104, generator=g, dtype=torch.float64)
    B = torch.randn(256, 4104, generator=g, dtype=torch.float64)
    C = torch.empty(256, 256, device=gpu)
    strided_gemm(A.float().to(gpu), B.float().to(gpu), C, M=256, N=256, K=4104, lda=4104, ldb=4104, ldc=256, path=4)
    ref = A.float().double() @ B.float().double().t()
    assert _rel_fro(C.cpu(), ref) <= 2e-5


def test_fp32_default_is_exact_non_integer(gpu):
    """the distributed products' fp32 GEMMs run EXACT fp32 by default (XDOT_FP32_MODE
    unset), checked on non-integer data against fp64 at torch-fp32 tolerance -- a split-bf16
    route (~1e-5) would fail this bound; split runs only when asked for."""
    from xdot.ops.gemm import strided_gemm
    from xdot.utils.env import FLAGS

    g = torch.Generator(device="cpu").manual_seed(11)
    M, N, K = 1024, 1024, 2048
    A = torch.randn(M, K, generator=g, dtype=torch.float64)
    B = torch.randn(N, K, generator=g, dtype=torch.float64)
    ref = A.float().double() @ B.float().double().t()
    old = FLAGS.fp32_mode
    try:
        FLAGS.fp32_mode = "exact"
        C = torch.empty(M, N, device=gpu)
        strided_gemm(A.float().to(gpu), B.float().to(gpu), C, M=M, N=N, K=K, lda=K, ldb=K, ldc=N)
        assert _rel_fro(C.cpu(), ref) <= 2e-6
        FLAGS.fp32_mode = "split"
        C2 = torch.empty(M, N, device=gpu)
        strided_gemm(A.float().to(gpu), B.float().to(gpu), C2, M=M, N=N, K=K, lda=K, ldb=K, ldc=N)
        assert _rel_fro(C2.cpu(), ref) <= 2e-5
    finally:
        FLAGS.fp32_mode = old


def test_split_fp32_non_finite_inputs(gpu):
    """split3: an inf operand gives inf (not NaN) products; |x| near FLT_MAX stays finite in hi/lo."""
    from xdot.ops.gemm import strided_gemm

    M = N = 256
    K = 64
    A = torch.ones(M, K, device=gpu)
    B = torch.full((N, K), 1e-3, device=gpu)
    A[3, 5] = float("inf")
    A[7, 9] = 3.3e38  # rounds to +inf in bf16: hi must be truncated instead
    C = torch.empty(M, N, device=gpu)
    strided_gemm(A, B, C, M=M, N=N, K=K, lda=K, ldb=K, ldc=N, path=4)
    ref = (A.double().cpu() @ B.double().cpu().t())
    assert torch.isinf(C[3]).all() and not torch.isnan(C).any()
    ok = torch.ones(M, dtype=torch.bool)
    ok[3] = False
    assert torch.allclose(C.cpu().double()[ok], ref[ok], rtol=2e-5, atol=1e-6)


@pytest.mark.parametrize("a_mc,b_mc", LAYOUTS)
@pytest.mark.parametrize("K", [4096, 5000])
def test_exact_fp32_k_slabs(gpu, a_mc, b_mc, K):
    """Exact fp32 with few output tiles and a long K runs as K slabs of the 128x128 kernel
    (fp32 partials + one ordered sum; a short last slab when the slab length does not divide
    K): exact-fp32 accuracy vs fp64, alpha / beta applied once."""
    from xdot.ops.gemm import strided_gemm
    from xdot.utils.env import FLAGS

    g = torch.Generator(device="cpu").manual_seed(K)
    M, N, nb = 300, 200, 2
    A = torch.randn(nb, *((K, M) if a_mc else (M, K)), generator=g, dtype=torch.float64)
    B = torch.randn(nb, *((K, N) if b_mc else (N, K)), generator=g, dtype=torch.float64)
    C0 = torch.randn(nb, M, N, generator=g, dtype=torch.float64)
    C = C0.float().to(gpu)
    old = FLAGS.fp32_mode
    try:
        FLAGS.fp32_mode = "exact"
        strided_gemm(A.float().to(gpu), B.float().to(gpu), C, M=M, N=N, K=K, nb2=nb, lda=(M if a_mc else K),
                     ldb=(N if b_mc else K), ldc=N, sA2=M * K, sB2=N * K, sC2=M * N, a_mc=a_mc, b_mc=b_mc,
                     alpha=0.5, beta=2.0)
    finally:
        FLAGS.fp32_mode = old
    Af, Bf = A.float().double(), B.float().double()
    opA = Af.transpose(-1, -2) if a_mc else Af
    opB = Bf if b_mc else Bf.transpose(-1, -2)
    ref = 0.5 * torch.matmul(opA, opB) + 2.0 * C0.float().double()
    assert _rel_fro(C.cpu(), ref) <= 2e-6
