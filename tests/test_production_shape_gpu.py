"""The kernels at the benchmark's own shapes: H = 8, D = 96, T = 25000.

* N = 1: R = T = 25000 through the flash kernels exactly as the module calls them (bf16 with the
  pre-scaled row side, exact fp32 with the score buffer): the head-heavy forward grid, the auto
  column splits of the row-side kernel and the 196-block column grid at real size.  A dense
  reference would need 20 GB of fp32 scores per tensor, so rows and columns of every head are
  SAMPLED and recomputed in fp64 (the pattern of tests/test_long_context_gpu.py).
* N = 8 rank: R = 3125 rows against T = 25000 through :class:`SeqParallelAttention` on an
  :class:`EmulatedComm` (rank 3 of 8: two gather chunks, own block first, the merged middle-rank
  segment plan, the chunk-permuted backward; fp32 takes the one-kernel score-buffer path): the
  emulated gather replicates the local shard, so the reference is dense attention against the
  shard repeated 8 times, and the reduce-scatter hands back block 3 of the gathered gradient.
  Matches tests/test_gradient.py's reference pattern (reference: tests/test_gradient.py:77-121).
"""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

H, D = 8, 96
C = H * D


def _rel(a, b):
    return ((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30)).item()


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_flash_n1_production_shape_sampled(gpu, dtype):
    from xdot.ops import flash

    R = T = 25_000
    scale = 1.0 / math.sqrt(D)
    g = torch.Generator(device=gpu).manual_seed(2500)
    rows = torch.randn(1, R, C, device=gpu, generator=g).to(dtype)
    qv = torch.randn(1, T, 2 * C, device=gpu, generator=g).to(dtype)  # packed [q | v] as the module
    do = torch.randn(1, R, C, device=gpu, generator=g).to(dtype)
    kc, vc = qv[..., :C], qv[..., C:]
    if dtype == torch.float32:
        sb = flash.score_buffer(1, H, R, T, gpu)
        assert sb is not None, "the 20 GB score buffer should fit an MI355X"
        out, lse = flash.fwd(rows, kc, vc, None, H, scale, fp32_mode=0, sbuf=sb)
        delta, lse2 = flash.bwd_prep(do, out, lse, H)
        dkv, _ = flash.bwd_cols(do, rows, kc, vc, out, lse, None, H, scale, delta, lse2=lse2, fp32_mode=0, sbuf=sb)
        drows = flash.bwd_rows(do, rows, kc, vc, lse, delta, None, H, scale, fp32_mode=0, sbuf=sb)
        tol = dict(o=1e-5, dr=2e-5, dc=2e-5, lse=1e-4)  # fp32 sums over 25000 columns
    else:
        rk = flash.prescale(rows, scale)
        out, lse = flash.fwd(rk, kc, vc, None, H, scale, prescaled=True)
        delta, lse2 = flash.bwd_prep(do, out, lse, H)
        dkv, _ = flash.bwd_cols(do, rk, kc, vc, out, lse, None, H, scale, delta, prescaled=True, lse2=lse2)
        drows = flash.bwd_rows(do, rk, kc, vc, lse, delta, None, H, scale, prescaled=True)
        tol = dict(o=2e-2, dr=3e-2, dc=3e-2, lse=5e-3)  # bf16-rounded prescaled rows
    torch.cuda.synchronize()
    for h in range(H):
        sl = slice(h * D, (h + 1) * D)
        Q, K, V, dO = rows[0, :, sl].double(), kc[0, :, sl].double(), vc[0, :, sl].double(), do[0, :, sl].double()
        ri = torch.randint(0, R, (24,), device=gpu, generator=g)
        s = (Q[ri] @ K.t()) * scale
        lse_ref = torch.logsumexp(s, -1)
        p = torch.exp(s - lse_ref[:, None])
        o_ref = p @ V
        assert _rel(out[0, ri, sl], o_ref) <= tol["o"], f"head {h} out"
        assert (lse[0, h, ri].double() - lse_ref).abs().max().item() < tol["lse"]
        dref = (dO[ri] * o_ref).sum(-1)
        ds = p * ((dO[ri] @ V.t()) - dref[:, None])
        assert _rel(drows[0, ri, sl], scale * (ds @ K)) <= tol["dr"], f"head {h} d rows"
        cj = torch.randint(0, T, (24,), device=gpu, generator=g)
        sc = (Q @ K[cj].t()) * scale                                       # (R, 24)
        lse_all = torch.logsumexp((Q @ K.t()) * scale, -1) if h == 0 else None
        if lse_all is not None:  # the LSE of every row, once (head 0): the kernel's own
            assert (lse[0, 0].double() - lse_all).abs().max().item() < tol["lse"]
        pc = torch.exp(sc - lse[0, h].double()[:, None])
        dsc = pc * ((dO @ V[cj].t()) - delta[0, h].double()[:, None])
        assert _rel(dkv[0, cj, C + h * D:C + (h + 1) * D], pc.t() @ dO) <= tol["dc"], f"head {h} dv"
        assert _rel(dkv[0, cj, sl], scale * (dsc.t() @ Q)) <= tol["dc"], f"head {h} dq"


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_seq_parallel_n8_rank_shape(gpu, dtype):
    from xdot.parallel.attention import SeqParallelAttention, _row_chunks
    from xdot.utils.comm import EmulatedComm

    n, rank, R = 8, 3, 3125
    T = n * R
    assert len(_row_chunks(n, R, True)) == 2  # the N=8 default gather pipeline
    comm = EmulatedComm(n, rank)
    scale = 1.0 / math.sqrt(D)
    g = torch.Generator(device=gpu).manual_seed(8)
    k = torch.randn(1, R, C, device=gpu, generator=g).to(dtype).requires_grad_(True)
    qv = torch.randn(1, R, 2 * C, device=gpu, generator=g).to(dtype).requires_grad_(True)
    mask = torch.rand(1, R, T, device=gpu, generator=g) < 0.1
    mask[..., rank * R] = False
    do = torch.randn(1, R, C, device=gpu, generator=g).to(dtype)
    out = SeqParallelAttention.apply(k, qv, mask, H, scale, comm)
    out.backward(do)

    kd = k.detach().double().view(1, R, H, D).transpose(1, 2).requires_grad_(True)
    full = qv.detach().double().repeat(1, n, 1).requires_grad_(True)     # what the emulated gather holds
    q = full[..., :C].reshape(1, T, H, D).transpose(1, 2)
    v = full[..., C:].reshape(1, T, H, D).transpose(1, 2)
    s = (kd @ q.transpose(-1, -2)) * scale
    s = s.masked_fill(mask.unsqueeze(1), -float("inf"))
    o = (torch.softmax(s, -1) @ v).transpose(1, 2).reshape(1, R, C)
    o.backward(do.double())
    dqv_ref = full.grad[:, rank * R:(rank + 1) * R]                       # the reduce-scatter's block
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-5
    assert _rel(out, o) <= tol
    assert _rel(k.grad, kd.grad.transpose(1, 2).reshape(1, R, C)) <= 1.5 * tol
    assert _rel(qv.grad, dqv_ref) <= 1.5 * tol
