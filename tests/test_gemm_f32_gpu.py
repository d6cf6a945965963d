"""Exact-fp32 GEMM (csrc/gemm_f32.hip) through ``xdot.gemm`` vs an fp64 torch reference (GPU).

The reference computes every distributed product in fp32 (multiplication/functions.py:96,142,209);
these products and the module's fp32 projections run this kernel by default (no library GEMM).
Bounds: relative Frobenius <= 2e-6 (an fp32 fmaf chain over K); integer-valued operands exact."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return ((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30)).item()


def _op(t, mc):
    return t.t() if mc else t


@pytest.mark.parametrize("a_mc", [False, True])
@pytest.mark.parametrize("b_mc", [False, True])
@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (300, 200, 97), (129, 1000, 33), (64, 31, 5), (1024, 768, 2048)])
def test_gemm_f32_layouts(gpu, a_mc, b_mc, M, N, K):
    from xdot.ops.gemm import strided_gemm

    g = torch.Generator(device=gpu).manual_seed(M + N + K)
    # storage: A(m, k) = A[m*lda + k] (k-contiguous) or A[k*lda + m]; B(k, n) = B[n*ldb + k] or B[k*ldb + n]
    A = torch.randn((K, M) if a_mc else (M, K), device=gpu, generator=g)
    B = torch.randn((K, N) if b_mc else (N, K), device=gpu, generator=g)
    C = torch.randn(M, N, device=gpu, generator=g)
    C0 = C.clone()
    strided_gemm(A, B, C, M=M, N=N, K=K, lda=A.shape[1], ldb=B.shape[1], ldc=N, a_mc=a_mc, b_mc=b_mc,
                 alpha=0.5, beta=-2.0)
    opA = A.double().t() if a_mc else A.double()
    opB = B.double() if b_mc else B.double().t()
    ref = 0.5 * opA @ opB - 2.0 * C0.double()
    assert _rel(C, ref) <= 2e-6


def _eligible_v2(M, N, K, a_mc, b_mc):
    return (a_mc or K % 4 == 0) and (b_mc or K % 4 == 0) and (not a_mc or M % 4 == 0) and (not b_mc or N % 4 == 0)


@pytest.mark.parametrize("a_mc", [False, True])
@pytest.mark.parametrize("b_mc", [False, True])
@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (300, 200, 100), (516, 1000, 36), (64, 36, 4), (1024, 768, 2048),
                                   (768, 520, 12500)])
def test_gemm2_f32_layouts(gpu, a_mc, b_mc, M, N, K):
    """The persistent 256x256 LDS-DMA kernel (path 2, csrc/gemm2_f32.hip): ragged M / N tiles,
    K tails (K % 32) zero-patched in LDS, alpha / beta, every storage order; the long-K shape
    goes split-K through path 0 (ordered fp32 partial sum)."""
    from xdot.ops.gemm import strided_gemm

    if not _eligible_v2(M, N, K, a_mc, b_mc):
        pytest.skip("layout rules of the 256x256 kernel")
    g = torch.Generator(device=gpu).manual_seed(M * 7 + N + K)
    A = torch.randn((K, M) if a_mc else (M, K), device=gpu, generator=g)
    B = torch.randn((K, N) if b_mc else (N, K), device=gpu, generator=g)
    C = torch.randn(M, N, device=gpu, generator=g)
    C0 = C.clone()
    path = 0 if K > 4096 else 2
    strided_gemm(A, B, C, M=M, N=N, K=K, lda=A.shape[1], ldb=B.shape[1], ldc=N, a_mc=a_mc, b_mc=b_mc,
                 alpha=0.5, beta=-2.0, path=path)
    opA = A.double().t() if a_mc else A.double()
    opB = B.double() if b_mc else B.double().t()
    assert _rel(C, 0.5 * opA @ opB - 2.0 * C0.double()) <= 2e-6


def test_gemm2_f32_batched_segments_exact_ints(gpu):
    """Two batch levels + K segments with a K tail per segment (K = 36) on the 256x256 kernel and
    through the automatic route (split-K): integer data, exact."""
    from xdot.ops.gemm import strided_gemm

    g = torch.Generator(device=gpu).manual_seed(3)
    nb1, nb2, nseg, M, N, K = 2, 2, 3, 260, 132, 36
    A = torch.randint(-3, 4, (nb1, nb2, nseg, K, M), device=gpu, generator=g).float()  # mn-contiguous
    B = torch.randint(-3, 4, (nb1, nb2, nseg, N, K), device=gpu, generator=g).float()  # k-contiguous
    ref = torch.einsum("xyskm,xysnk->xymn", A.double(), B.double())
    for path in (2, 0):
        C = torch.full((nb1, nb2, M, N), float("nan"), device=gpu)
        strided_gemm(A, B, C, M=M, N=N, K=K, nseg=nseg, nb1=nb1, nb2=nb2, lda=M, ldb=K, ldc=N,
                     sA1=nb2 * nseg * K * M, sA2=nseg * K * M, sB1=nb2 * nseg * N * K, sB2=nseg * N * K,
                     sC1=nb2 * M * N, sC2=M * N, sAseg=K * M, sBseg=N * K, a_mc=True, path=path)
        assert torch.equal(C.double(), ref), f"path {path}"


def test_gemm_f32_batched_segments_exact_ints(gpu):
    """2-level batch + K segments (the `all` product's rank segments) on integer data: exact."""
    from xdot.ops.gemm import strided_gemm

    g = torch.Generator(device=gpu).manual_seed(0)
    nb1, nb2, nseg, M, N, K = 2, 3, 4, 130, 70, 45
    A = torch.randint(-3, 4, (nb1, nb2, nseg, M, K), device=gpu, generator=g).float()
    B = torch.randint(-3, 4, (nb1, nb2, nseg, K, N), device=gpu, generator=g).float()
    C = torch.empty(nb1, nb2, M, N, device=gpu)
    strided_gemm(A, B, C, M=M, N=N, K=K, nseg=nseg, nb1=nb1, nb2=nb2, lda=K, ldb=N, ldc=N,
                 sA1=nb2 * nseg * M * K, sA2=nseg * M * K, sB1=nb2 * nseg * K * N, sB2=nseg * K * N,
                 sC1=nb2 * M * N, sC2=M * N, sAseg=M * K, sBseg=K * N, b_mc=True)
    ref = torch.einsum("xysmk,xyskn->xymn", A.double(), B.double())
    assert torch.equal(C.double(), ref)


def test_gemm_f32_long_k_slabs(gpu):
    """Few output tiles and a long K (the weight gradients, the autograd ops' K = T products):
    K slabs of the kernel + one ordered sum."""
    from xdot.ops.gemm import strided_gemm

    g = torch.Generator(device=gpu).manual_seed(1)
    M, N, K = 768, 768, 25000
    A = torch.randn(K, M, device=gpu, generator=g)
    B = torch.randn(K, N, device=gpu, generator=g)
    C = torch.empty(M, N, device=gpu)
    strided_gemm(A, B, C, M=M, N=N, K=K, lda=M, ldb=N, ldc=N, a_mc=True, b_mc=True)
    assert _rel(C, A.double().t() @ B.double()) <= 2e-6


def test_fp32_projections_native(gpu):
    """fp32 Linear forward / input grad / weight grad (xdot.ops.linear) on the exact kernel."""
    from xdot.ops.linear import linear

    g = torch.Generator(device=gpu).manual_seed(2)
    x = torch.randn(3, 333, 256, device=gpu, generator=g, requires_grad=True)
    w = torch.randn(192, 256, device=gpu, generator=g, requires_grad=True)
    b = torch.randn(192, device=gpu, generator=g, requires_grad=True)
    y = linear(x, w, b)
    dy = torch.randn_like(y)
    y.backward(dy)
    xd, wd, bd = (t.detach().double().requires_grad_(True) for t in (x, w, b))
    yr = torch.nn.functional.linear(xd, wd, bd)
    yr.backward(dy.double())
    assert _rel(y, yr) <= 2e-6
    for got, ref in ((x.grad, xd.grad), (w.grad, wd.grad), (b.grad, bd.grad)):
        assert _rel(got, ref) <= 2e-6
