"""Numerics of the 256x256 LDS-DMA GEMM (csrc/gemm2.hip) against fp32 PyTorch (GPU only).

Every call forces the v2 path (``path=2``; 16-bit operands, aligned layouts): every operand layout, M/N/K tails, K segments, split-K, alpha/beta.
"""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

HALF = [torch.bfloat16, torch.float16]


def _tol(dt, k):
    return (2e-2 if dt == torch.bfloat16 else 4e-3) * math.sqrt(max(k, 1) / 64)


def _run(gpu, dt, a_mc, b_mc, M, N, K, nseg=1, batches=2, alpha=1.0, beta=0.0, out_dt=torch.float32, seed=0):
    from xdot.ops.gemm import strided_gemm

    g = torch.Generator(device="cpu").manual_seed(seed + M * 7 + N + K)
    A = torch.randn(batches, nseg, *((K, M) if a_mc else (M, K)), generator=g).to(gpu, dt)
    B = torch.randn(batches, nseg, *((K, N) if b_mc else (N, K)), generator=g).to(gpu, dt)
    C0 = torch.randn(batches, M, N, generator=g).to(gpu, out_dt)
    C = C0.clone()
    strided_gemm(A, B, C, M=M, N=N, K=K, nseg=nseg, nb2=batches, lda=(M if a_mc else K),
                 ldb=(N if b_mc else K), ldc=N, sA2=nseg * M * K, sB2=nseg * N * K, sC2=M * N,
                 sAseg=M * K, sBseg=N * K, a_mc=a_mc, b_mc=b_mc, alpha=alpha, beta=beta, path=2)
    Af, Bf = A.float(), B.float()
    opA = Af.transpose(-1, -2) if a_mc else Af        # (b, s, M, K)
    opB = Bf if b_mc else Bf.transpose(-1, -2)        # (b, s, K, N)
    ref = alpha * torch.matmul(opA, opB).sum(1) + beta * C0.float()
    err = (C.float() - ref).abs().max().item()
    tol = _tol(dt, K * nseg) * max(1.0, ref.abs().max().item() / 4)
    if out_dt != torch.float32:
        tol += ref.abs().max().item() * (2 ** -7 if out_dt == torch.bfloat16 else 2 ** -10)
    assert err <= tol, (err, tol)


@pytest.mark.parametrize("dt", HALF)
@pytest.mark.parametrize("a_mc,b_mc", [(False, False), (False, True), (True, False), (True, True)])
@pytest.mark.parametrize("M,N,K", [(256, 256, 32), (520, 264, 96), (776, 1000, 40), (264, 520, 200)])
def test_gemm2_layouts_tails(gpu, dt, a_mc, b_mc, M, N, K):
    _run(gpu, dt, a_mc, b_mc, M, N, K, alpha=0.5)


@pytest.mark.parametrize("a_mc,b_mc", [(False, False), (False, True), (True, False), (True, True)])
def test_gemm2_segments_beta_bf16_out(gpu, a_mc, b_mc):
    _run(gpu, torch.bfloat16, a_mc, b_mc, 512, 264, 104, nseg=3, alpha=0.25, beta=1.0, out_dt=torch.bfloat16)


@pytest.mark.parametrize("a_mc,b_mc", [(False, False), (True, True), (False, True)])
@pytest.mark.parametrize("K", [4096, 4104])
def test_gemm2_split_k(gpu, a_mc, b_mc, K):
    """one 256x256 tile per batch and a long K: the dispatcher splits K (fp32 partials)"""
    _run(gpu, torch.bfloat16, a_mc, b_mc, 256, 256, K, batches=1, alpha=2.0, beta=0.5)


def test_gemm2_nt_distributed_product(gpu):
    """the nt product through the op-level helper (final (P, R, T) layout, automatic kernel choice)"""
    from xdot.ops.gemm import nt_chunk_into

    N, Pn, R, D = 3, 2, 320, 96
    left = torch.randn(Pn, R, D, device=gpu).bfloat16()
    chunk = torch.randn(N, Pn, R, D, device=gpu).bfloat16()
    out = torch.empty(Pn, R, N * R, device=gpu, dtype=torch.bfloat16)
    nt_chunk_into(out, left, chunk, 0, alpha=0.125)
    ref = 0.125 * torch.cat([left.float() @ chunk.float()[j].transpose(-1, -2) for j in range(N)], -1)
    assert torch.allclose(out.float(), ref, atol=0.05, rtol=2e-2)


@pytest.mark.parametrize("a_mc,b_mc", [(False, False), (True, True), (False, True), (True, False)])
def test_gemm2_persistent_many_items(gpu, a_mc, b_mc):
    """more work items than CUs: each persistent workgroup crosses item boundaries (edge tiles,
    K tails, segments) with the DMA ring running on"""
    _run(gpu, torch.bfloat16, a_mc, b_mc, 1288, 1800, 200, nseg=2, batches=5, alpha=0.5, beta=0.25,
         out_dt=torch.bfloat16)


def test_gemm2_split_k_many_items(gpu):
    _run(gpu, torch.float16, False, True, 264, 512, 6000, batches=6, alpha=1.0)


@pytest.mark.parametrize("K", [32, 64, 256])
@pytest.mark.parametrize("out_dt", [torch.bfloat16, torch.float32])
def test_gemm2_persistent_interior_items(gpu, K, out_dt):
    """interior 256x256 items only (uniform epilogue stores), more items than CUs, K % 32 == 0:
    short items put epilogues back to back while the ring keeps streaming"""
    _run(gpu, torch.bfloat16, False, False, 2304, 2560, K, batches=3, out_dt=out_dt)
    _run(gpu, torch.bfloat16, False, True, 2304, 2560, K, batches=3, out_dt=out_dt)


def test_gemm_library_route_matches_kernels(gpu):
    """large plain products through the op-level helpers (gemm3 by default; with
    XDOT_GEMM_LIB=1 the library route on in-place strided views, one batch level, merged K
    segments, tn's interleaved column blocks of `left` against one broadcast `right`); nt's
    per-rank column blocks interleaved in one output row stay on the xdot kernels either way --
    all must agree with torch on the same data"""
    from xdot.ops.gemm import all_chunk_into, nt_chunk_into, tn_partials_into

    g = torch.Generator(device="cpu").manual_seed(5)
    N, Pn, R, D = 2, 2, 2048, 128
    T = N * R
    left = torch.randn(Pn, R, D, generator=g).to(gpu, torch.bfloat16)
    chunk = torch.randn(N, Pn, R, D, generator=g).to(gpu, torch.bfloat16)
    out = torch.empty(Pn, R, T, device=gpu, dtype=torch.bfloat16)
    nt_chunk_into(out, left, chunk, 0)                      # nb1 = N, nb2 = Pn: merged batch? (no: sC1 = Rr)
    ref = torch.cat([left.float() @ chunk.float()[j].transpose(-1, -2) for j in range(N)], -1)
    assert torch.allclose(out.float(), ref, atol=0.1, rtol=2e-2)

    # plain nt (N = 1): one batched GEMM over heads, output (Pn, R, T) in place
    T1 = 16384
    left1 = torch.randn(1, 4096, 256, generator=g).to(gpu, torch.bfloat16)
    chunk1 = torch.randn(1, 1, T1, 256, generator=g).to(gpu, torch.bfloat16)
    out1 = torch.empty(1, 4096, T1, device=gpu, dtype=torch.bfloat16)
    nt_chunk_into(out1, left1, chunk1, 0, alpha=0.5)
    ref1 = 0.5 * (left1.float() @ chunk1.float()[0].transpose(-1, -2))
    assert torch.allclose(out1.float(), ref1, atol=0.25, rtol=2e-2)

    # all with K segments that continue each other (merged into one K = T GEMM)
    leftA = torch.randn(1, 4096, 4 * 4096, generator=g).to(gpu, torch.bfloat16) / 64
    chunkA = torch.randn(4, 1, 4096, 1024, generator=g).to(gpu, torch.bfloat16)
    outA = torch.empty(1, 4096, 1024, device=gpu, dtype=torch.bfloat16)
    all_chunk_into(outA, leftA, chunkA, 0)
    refA = sum(leftA.float()[..., j * 4096:(j + 1) * 4096] @ chunkA.float()[j] for j in range(4))
    assert torch.allclose(outA.float(), refA, atol=0.1, rtol=2e-2)

    # tn partials: N blocks (nb1 = N) of leftᵀ @ right
    leftT = torch.randn(1, 4096, 2 * 4096, generator=g).to(gpu, torch.bfloat16) / 64
    rightT = torch.randn(1, 4096, 1024, generator=g).to(gpu, torch.bfloat16)
    send = torch.empty(2, 1, 4096, 1024, device=gpu, dtype=torch.bfloat16)
    tn_partials_into(send, leftT, rightT)
    refT = torch.stack([leftT.float()[..., j * 4096:(j + 1) * 4096].transpose(-1, -2) @ rightT.float() for j in range(2)])
    assert torch.allclose(send.float(), refT, atol=0.1, rtol=2e-2)


def test_nt_rank_blocks_at_eight_ranks(gpu):
    """nt's eight per-rank column blocks of a (1, R, T) output (broadcast left, interleaved
    output batches, odd R = 3125): the layout that must stay off the library GEMM route; and the
    whole-shard case as one GEMM over all T columns"""
    from xdot.ops.gemm import nt_chunk_into

    g = torch.Generator(device="cpu").manual_seed(9)
    N, R, D = 8, 3125, 768
    left = torch.randn(1, R, D, generator=g).to(gpu, torch.bfloat16)
    chunk = torch.randn(N, 1, R, D, generator=g).to(gpu, torch.bfloat16)
    out = torch.empty(1, R, N * R, device=gpu, dtype=torch.bfloat16)
    h = 1563  # two row chunks per shard: per-rank column blocks (the whole-shard case is one GEMM)
    nt_chunk_into(out, left, chunk[:, :, :h], 0, alpha=0.25)
    nt_chunk_into(out, left, chunk[:, :, h:], h, alpha=0.25)
    torch.cuda.synchronize()
    rows = torch.arange(0, R, 311)
    ref = 0.25 * (left[0, rows].float() @ chunk[:, 0].float().reshape(N * R, D).t())
    assert torch.allclose(out[0, rows].float(), ref, atol=0.15, rtol=2e-2)
    out2 = torch.empty_like(out)
    nt_chunk_into(out2, left, chunk, 0, alpha=0.25)
    assert torch.allclose(out2[0, rows].float(), ref, atol=0.15, rtol=2e-2)
