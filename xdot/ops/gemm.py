"""Python face of the generic MFMA GEMM (``csrc/gemm.hip``).

``strided_gemm`` exposes the kernel's full addressing model (2-level batch, K segments,
either operand k- or mn-contiguous); the helpers below express the three distributed
products of the reference with it.  Every helper also has a torch reference path used on
CPU, for dtypes the kernel does not take (float64 / integer) and for testing.
"""
from __future__ import annotations

from typing import Optional

import torch

from .. import _ext
from ..utils.env import FLAGS

_HIP_IN = (torch.bfloat16, torch.float16, torch.float32)


def hip_dtype_ok(*ts: torch.Tensor) -> bool:
    return all(t.dtype in _HIP_IN for t in ts) and len({t.dtype for t in ts}) == 1


def strided_gemm(A, B, C, *, M, N, K, nseg=1, nb1=1, nb2=1, lda, ldb, ldc, sA1=0, sA2=0,
                 sB1=0, sB2=0, sC1=0, sC2=0, sAseg=0, sBseg=0, a_mc=False, b_mc=False,
                 alpha=1.0, beta=0.0, path=0, split_ok=True) -> None:
    """C[z1, z2](m, n) = alpha * sum_s sum_k opA(m, k) * opB(k, n) + beta * C[z1, z2](m, n)
    (csrc/gemm.hip; 16-bit operands with large outputs run the 256x256 csrc/gemm2.hip).

    ``path``: 0 = automatic kernel choice, 1 = the 128x128 kernel, 2 = the 256x256 kernel, 3 = the 8-phase
    16x16x32 kernel (raises if it declines), 4 = fp32 as three bf16 products on it, 5 = the 8-phase kernel
    where it takes the call, else the 256x256 one -- whenever the layout rules hold; 6 = automatic
    with the split-fp32 route allowed (what path 0 becomes for fp32 operands under
    ``XDOT_FP32_MODE=split``; the default ``exact`` keeps fp32 products on the exact fp32 MFMA kernel).
    ``FLAGS.fp32_mode`` is read here on every call: the one source of truth for the GEMMs too.
    ``split_ok=False`` keeps an fp32 call on the exact kernels under either mode."""
    if path == 0 and split_ok and A.dtype == torch.float32 and FLAGS.fp32_mode == "split":
        path = 6
    _ext.ops().gemm(A, B, C, int(M), int(N), int(K), int(nseg), int(nb1), int(nb2), int(lda),
                    int(ldb), int(ldc), int(sA1), int(sA2), int(sB1), int(sB2), int(sC1), int(sC2),
                    int(sAseg), int(sBseg), bool(a_mc), bool(b_mc), float(alpha),
                    float(beta), int(path))


def _flat(t: torch.Tensor, lead: int) -> torch.Tensor:
    """contiguous view with the leading ``lead`` dims flattened to one"""
    t = t.contiguous()
    return t.view(-1, *t.shape[t.dim() - lead:]) if lead else t


def _m3(x: torch.Tensor):
    """(Pn, rows, cols) operand read in place: -> (tensor, batch stride, row stride) when its
    inner stride is 1 (e.g. the (1, H, R, d) head-split view of a (1, R, H*d) projection, batch
    stride d, row stride H*d: no head-transpose copy), else a contiguous copy."""
    if x.dim() == 3 and (x.stride(-1) == 1 or x.shape[-1] == 1):
        P, r, c = x.shape
        return x, (x.stride(0) if P > 1 else 0), (x.stride(1) if r > 1 else c)
    x = x.contiguous()
    return x, x.shape[1] * x.shape[2], x.shape[2]


def _m4(x: torch.Tensor):
    """(N, Pn, rows, cols) operand in place -> (tensor, stride N, stride Pn, row stride)."""
    if x.stride(-1) == 1 or x.shape[-1] == 1:
        N, P, r, c = x.shape
        return x, (x.stride(0) if N > 1 else 0), (x.stride(1) if P > 1 else 0), (x.stride(2) if r > 1 else c)
    x = x.contiguous()
    return x, x.shape[1] * x.shape[2] * x.shape[3], x.shape[2] * x.shape[3], x.shape[3]


# ---------------------------------------------------------------------------------------
# nt: out[p, :, j*R + c0 : j*R + c0 + c] = alpha * left[p] @ chunk[j, p]^T
# ---------------------------------------------------------------------------------------
def nt_chunk_into(out: torch.Tensor, left: torch.Tensor, chunk: torch.Tensor, c0: int,
                  alpha: float = 1.0) -> None:
    """``out``: (Pn, R, N*Rr) contiguous; ``left``: (Pn, R, D); ``chunk``: (N, Pn, c, D); the
    operands may be strided views with unit inner stride (read in place)."""
    N, Pn, c, D = chunk.shape
    R = left.shape[-2]
    T = out.shape[-1]
    Rr = T // N  # rows per rank of the gathered operand
    if _ext.use_hip(out, left, chunk) and hip_dtype_ok(left, chunk) and out.dtype in _HIP_IN:
        left, sA, lda = _m3(left)
        chunk, sBj, sBp, ldb = _m4(chunk)
        if N > 1 and c0 == 0 and c == Rr and sBj == Rr * ldb:
            # whole shards whose rank blocks continue each other along the rows (rank-major
            # gather, or the R-major head-split gather): ONE GEMM over all T columns.  Per-rank
            # column blocks would start off 16-byte boundaries whenever T/N is odd (R = 3125:
            # 7 of 8 blocks) and fall back to element stores (measured 1.23 ms vs one GEMM)
            strided_gemm(left, chunk, out, M=R, N=T, K=D, nb2=Pn, lda=lda, ldb=ldb, ldc=T, sA2=sA, sB2=sBp,
                         sC2=R * T, a_mc=False, b_mc=False, alpha=alpha)
            return
        strided_gemm(left, chunk, out[..., c0:], M=R, N=c, K=D, nb1=N, nb2=Pn,
                     lda=lda, ldb=ldb, ldc=T, sA1=0, sA2=sA, sB1=sBj, sB2=sBp,
                     sC1=Rr, sC2=R * T, a_mc=False, b_mc=False, alpha=alpha)
        return
    part = torch.matmul(left.unsqueeze(0).to(torch.promote_types(left.dtype, chunk.dtype)),
                        chunk.transpose(-1, -2))                      # (N, Pn, R, c)
    if alpha != 1.0:
        part = part * alpha
    ov = out.view(Pn, R, N, Rr)
    ov[..., c0:c0 + c] = part.permute(1, 2, 0, 3).to(out.dtype)


def nt_block_into(out: torch.Tensor, left: torch.Tensor, blk: torch.Tensor, alpha: float = 1.0) -> None:
    """``out[p] = alpha * left[p] @ blk[p]ᵀ``: (Pn, R, D) x (Pn, c, D) -> (Pn, R, c).  Every operand
    may be a strided view with unit inner stride (``out``: e.g. one source rank's column block
    of the (Pn, R, T) ``nt`` result, written in place by the ring schedule)."""
    Pn, R, D = left.shape
    c = blk.shape[-2]
    if _ext.use_hip(out, left, blk) and hip_dtype_ok(left, blk) and out.dtype in _HIP_IN:
        a, sA, lda = _m3(left)
        b, sB, ldb = _m3(blk)
        o, sC, ldc = _m3(out)
        strided_gemm(a, b, o, M=R, N=c, K=D, nb2=Pn, lda=lda, ldb=ldb, ldc=ldc, sA2=sA, sB2=sB, sC2=sC,
                     a_mc=False, b_mc=False, alpha=alpha)
        if o is not out:
            out.copy_(o)
        return
    ct = torch.promote_types(left.dtype, blk.dtype)
    r = torch.matmul(left.to(ct), blk.to(ct).transpose(-1, -2))
    if alpha != 1.0:
        r = r * alpha
    out.copy_(r.to(out.dtype))


# ---------------------------------------------------------------------------------------
# all: out[p, :, d0:d0+c] = sum_j left[p, :, j*R:(j+1)*R] @ chunk[j, p]
# ---------------------------------------------------------------------------------------
def all_chunk_into(out: torch.Tensor, left: torch.Tensor, chunk: torch.Tensor, d0: int) -> None:
    """``out``: (Pn, R, D); ``left``: (Pn, R, T); ``chunk``: (N, Pn, R, c) feature columns."""
    N, Pn, R, c = chunk.shape
    T = left.shape[-1]
    if _ext.use_hip(out, left, chunk) and hip_dtype_ok(left, chunk) and out.dtype in _HIP_IN:
        left, sA, lda = _m3(left)
        chunk, sBj, sBp, ldb = _m4(chunk)
        out_, sC, ldc = _m3(out)
        strided_gemm(left, chunk, out_[..., d0:], M=R, N=c, K=R, nseg=N, nb1=1, nb2=Pn,
                     lda=lda, ldb=ldb, ldc=ldc, sA2=sA, sB2=sBp, sC2=sC,
                     sAseg=R, sBseg=sBj, a_mc=False, b_mc=True)
        if out_ is not out:  # _m3 made a contiguous temporary: write the columns back
            out[..., d0:d0 + c].copy_(out_[..., d0:d0 + c])
        return
    ct = torch.promote_types(left.dtype, chunk.dtype)
    splits = left.reshape(Pn, R, N, R).permute(2, 0, 1, 3).to(ct)     # no stack copy
    res = torch.matmul(splits, chunk.to(ct)).sum(0)                   # (Pn, R, c)
    out[..., d0:d0 + c] = res.to(out.dtype)


# ---------------------------------------------------------------------------------------
# all, row-block chunks: acc[p] (+)= sum_j left[p, :, j*R + r0 : j*R + r0 + c] @ chunk[j, p]
# ---------------------------------------------------------------------------------------
def all_rows_chunk_into(acc: torch.Tensor, left: torch.Tensor, chunk: torch.Tensor, r0: int, accumulate: bool) -> None:
    """``acc``: (Pn, R, D); ``left``: (Pn, R, T); ``chunk``: (N, Pn, c, D) = rows r0..r0+c of every
    rank's ``right``.  ``accumulate``: add to ``acc`` (beta = 1) instead of overwriting it."""
    N, Pn, c, D = chunk.shape
    R, T = left.shape[-2], left.shape[-1]
    Rr = T // N
    if _ext.use_hip(acc, left, chunk) and hip_dtype_ok(left, chunk) and acc.dtype in _HIP_IN:
        left, sA, lda = _m3(left)
        chunk, sBj, sBp, ldb = _m4(chunk)
        acc_, sC, ldc = _m3(acc)
        strided_gemm(left[..., r0:], chunk, acc_, M=R, N=D, K=c, nseg=N, nb1=1, nb2=Pn,
                     lda=lda, ldb=ldb, ldc=ldc, sA2=sA, sB2=sBp, sC2=sC,
                     sAseg=Rr, sBseg=sBj, a_mc=False, b_mc=True, beta=1.0 if accumulate else 0.0)
        if acc_ is not acc:
            acc.copy_(acc_)
        return
    ct = acc.dtype if acc.dtype in (torch.float32, torch.float64) else torch.float32
    part = sum(torch.matmul(left[..., j * Rr + r0:j * Rr + r0 + c].to(ct), chunk[j].to(ct)) for j in range(N))
    if accumulate:
        acc += part.to(acc.dtype)
    else:
        acc.copy_(part)


# ---------------------------------------------------------------------------------------
# tn: send[j, p] = left[p, :, j*R:(j+1)*R]^T @ right[p]   (reduce-scatter send buffer)
# ---------------------------------------------------------------------------------------
def tn_partials_into(send: torch.Tensor, left: torch.Tensor, right: torch.Tensor) -> None:
    """``send``: (N, Pn, R, D) (any view with unit inner stride, e.g. an (N, R, Pn, D) buffer
    permuted); ``left``: (Pn, R, T); ``right``: (Pn, R, D), read in place."""
    N, Pn, R, D = send.shape
    T = left.shape[-1]
    if _ext.use_hip(send, left, right) and hip_dtype_ok(left, right) and send.dtype in _HIP_IN:
        left, sA, lda = _m3(left)
        right, sB, ldb = _m3(right)
        assert send.stride(-1) == 1, "tn_partials_into: send needs a unit inner stride"
        sCj, sCp, ldc = send.stride(0), send.stride(1), send.stride(2)
        if (R * left.element_size()) % 16 and send.stride() == (R * Pn * D, D, Pn * D, 1):
            # R-major send buffer (n, R, Pn, D): rows t = j*R + r of head p are uniformly Pn*D apart,
            # so the single T-row GEMM below writes it in place
            T_ = N * R
            strided_gemm(left, right, send, M=T_, N=D, K=R, nb2=Pn, lda=lda, ldb=ldb, ldc=Pn * D, sA2=sA,
                         sB2=sB, sC2=D, a_mc=True, b_mc=True)
            return
        if (R * left.element_size()) % 16 and send.is_contiguous():
            # column blocks j*R of `left` start off 16-byte boundaries (odd T/N): ONE GEMM over all
            # T columns instead (leftᵀ (T x R) @ right, rows t = j*R + r), whose operand rows are aligned
            T_ = N * R
            dst = send.view(T_, D) if Pn == 1 else torch.empty(Pn, T_, D, dtype=send.dtype, device=send.device)
            strided_gemm(left, right, dst, M=T_, N=D, K=R, nb2=Pn, lda=lda, ldb=ldb, ldc=D, sA2=sA, sB2=sB,
                         sC2=T_ * D, a_mc=True, b_mc=True)
            if Pn > 1:
                send.copy_(dst.view(Pn, N, R, D).transpose(0, 1))
            return
        strided_gemm(left, right, send, M=R, N=D, K=R, nb1=N, nb2=Pn,
                     lda=lda, ldb=ldb, ldc=ldc, sA1=R, sA2=sA, sB1=0, sB2=sB,
                     sC1=sCj, sC2=sCp, a_mc=True, b_mc=True)
        return
    ct = torch.promote_types(left.dtype, right.dtype)
    blocks = left.reshape(Pn, R, N, R).permute(2, 0, 3, 1).to(ct)     # (N, Pn, R_col, R_row)
    send.copy_(torch.matmul(blocks, right.to(ct).unsqueeze(0)).to(send.dtype))


def matmul_into(out: torch.Tensor, a: torch.Tensor, b: torch.Tensor) -> None:
    """``out[p] = a[p] @ b[p]``: (Pn, M, K) x (Pn, K, N) -> (Pn, M, N); every operand may be a
    view with unit inner stride (read / written in place)."""
    Pn, M, K = a.shape
    N = b.shape[-1]
    if _ext.use_hip(out, a, b) and hip_dtype_ok(a, b) and out.dtype in _HIP_IN:
        a, sA, lda = _m3(a)
        b, sB, ldb = _m3(b)
        o, sC, ldc = _m3(out)
        strided_gemm(a, b, o, M=M, N=N, K=K, nb2=Pn, lda=lda, ldb=ldb, ldc=ldc, sA2=sA, sB2=sB,
                     sC2=sC, a_mc=False, b_mc=True)
        if o is not out:
            out.copy_(o)
        return
    ct = torch.promote_types(a.dtype, b.dtype)
    out.copy_(torch.matmul(a.to(ct), b.to(ct)))


def matmul(a: torch.Tensor, b: torch.Tensor, *, trans_b: bool = False, alpha: float = 1.0,
           out_dtype: Optional[torch.dtype] = None) -> torch.Tensor:
    """Batched ``alpha * a @ op(b)`` on the MFMA kernel (local, non-distributed helper)."""
    if not (_ext.use_hip(a, b) and hip_dtype_ok(a, b)):
        r = torch.matmul(a, b.transpose(-1, -2) if trans_b else b)
        return (r * alpha if alpha != 1.0 else r).to(out_dtype or r.dtype)
    lead = a.shape[:-2]
    a3 = _flat(a, 2)
    b3 = _flat(b, 2)
    if b3.shape[0] not in (1, a3.shape[0]):
        raise ValueError("matmul: batch mismatch")
    Pn, M, K = a3.shape
    N = b3.shape[-2] if trans_b else b3.shape[-1]
    out = torch.empty(Pn, M, N, dtype=out_dtype or a.dtype, device=a.device)
    sb = 0 if b3.shape[0] == 1 else b3.shape[-1] * b3.shape[-2]
    strided_gemm(a3, b3, out, M=M, N=N, K=K, nb2=Pn, lda=K, ldb=b3.shape[-1], ldc=N,
                 sA2=M * K, sB2=sb, sC2=M * N, a_mc=False, b_mc=not trans_b, alpha=alpha)
    return out.view(*lead, M, N)
