"""Projection ``Linear`` on xdot MFMA kernels: forward and input gradient on the projection GEMM
(``csrc/gemm_proj.hip``), split-K weight gradient on the GEMM kernels (``csrc/gemm2.hip``).

The four projections of the module (reference: ``distributed_dot_product/module.py:36-39``,
applied at ``:43-45`` and ``:75``) are ordinary ``nn.Linear`` layers.  Their forward
``y = x·Wᵀ + b`` and input gradient ``dX = dY·W`` (:func:`proj`, :func:`proj_dx`) pick a tile size
per shape so the T/N = 3125-row products of an N=8 rank still put >= 2 workgroups on every CU
(the library's host cost per call, ~19 µs, also exceeded its GPU time there:
``profiles/r3_rank_host.md``).  The weight gradient
``dW = dYᵀ·X`` has a reduction over the sequence (K = T/N rows: 25000 at N = 1)
while the output is only 768 x 768 (9 tiles of 256²) — hipBLASLt runs it at ≈170-330 TF/s
with most CUs idle.  Here K is split into slices that fill the 256 CUs (the 256x256 kernel of
``csrc/gemm2.hip`` chooses the split; other shapes use S slabs of the 128x128 kernel), each
slice writes an fp32 partial (bf16 inputs, fp32 accumulation), and one reduction sums them in
fp32 before the cast to the parameter dtype.

``linear(x, weight, bias)`` is a drop-in for ``torch.nn.functional.linear``; parameters stay
in the caller's ``nn.Linear`` modules (``state_dict`` compatible with the reference).
"""
from __future__ import annotations

import contextlib
from typing import Optional

import torch
import torch.nn.functional as F

from .. import _ext
from ..utils.env import FLAGS
from .gemm import strided_gemm

__all__ = ["linear", "linear_backward", "weight_grad", "weight_grad_pair", "LinearFn", "proj", "proj_dx"]

_SLOTS = 512       # 2 workgroups per CU x 256 CUs
_MIN_SLAB = 256    # rows of K per split
_WGRAD_PATH = 5    # gemm3 where it takes the shape (>= 256 x 256), else the 256x256 v2 kernel


def _splits(M: int, N: int, K: int) -> int:
    """K slabs: enough (tiles x S) workgroups to fill the GPU, >= _MIN_SLAB rows each; a
    divisor of K when one is at least a third of the target (no remainder launch)."""
    tiles = -(-M // 128) * -(-N // 128)
    s = max(1, min(-(-_SLOTS // tiles), K // _MIN_SLAB, 64))
    for d in range(s, max(1, s // 3) - 1, -1):
        if K % d == 0:
            return d
    return s


def _proj_ok(x: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor] = None) -> bool:
    from ..utils.env import FLAGS

    return (FLAGS.proj_kernel > 0 and x.dtype in (torch.bfloat16, torch.float16) and x.dtype == weight.dtype
            and (bias is None or bias.dtype == x.dtype) and _ext.use_hip(x, weight))


def _f32_ok(*ts) -> bool:
    """Exact-fp32 products of a projection on the exact-fp32 GEMM kernels (through xdot.gemm with
    split_ok off): fp32 GPU tensors, ``XDOT_F32_PROJ`` on (the library's fp32 GEMM otherwise).
    Under ``XDOT_FP32_MODE=split`` too: only the attention products take the split-bf16 route there
    (the library's fp32 projections cost the split step 4.3 ms against 2.6 on these kernels,
    profiles/r5_fp32.md), the projections stay exact."""
    return (FLAGS.f32_proj and all(t is None or (t.dtype == torch.float32 and t.is_cuda) for t in ts)
            and FLAGS.fp32_mode in ("exact", "split") and _ext.use_hip(*[t for t in ts if t is not None]))


def _force() -> int:
    from ..utils.env import FLAGS

    return 1 if FLAGS.proj_kernel >= 2 else 0


def proj(x: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor] = None,
         out: Optional[torch.Tensor] = None, alpha: float = 1.0) -> torch.Tensor:
    """``alpha * F.linear(x, weight, bias)`` on the projection GEMM (16-bit GPU tensors; shapes it
    does not take run on the library inside the op), rounded once.  ``out``: an (M, N) row-major
    view to write, e.g. this rank's block of an all-gather buffer."""
    if _proj_ok(x, weight, bias):
        return _ext.ops().proj(x, weight, bias, False, out, _force(), float(alpha))
    if _f32_ok(x, weight, bias):
        K = x.shape[-1]
        x2 = x.reshape(-1, K)
        if x2.stride(-1) != 1 or x2.stride(0) != K:
            x2 = x2.contiguous()
        w = weight.contiguous()
        M, N = x2.shape[0], w.shape[0]
        y = torch.empty(M, N, dtype=x.dtype, device=x.device) if out is None else out
        if bias is not None:
            y.copy_(bias.expand(M, N))  # C = alpha * x Wᵀ + alpha * bias
        strided_gemm(x2, w, y, M=M, N=N, K=K, lda=K, ldb=K, ldc=y.stride(0), alpha=alpha,
                     beta=alpha if bias is not None else 0.0, split_ok=False)
        return y if out is not None else y.view(*x.shape[:-1], N)
    if out is None:
        y = F.linear(x, weight, bias)
        return y if alpha == 1.0 else y.mul_(alpha)
    x2 = x.reshape(-1, x.shape[-1])
    if bias is None:
        torch.mm(x2, weight.t(), out=out)
        return out if alpha == 1.0 else out.mul_(alpha)
    return torch.addmm(bias, x2, weight.t(), beta=alpha, alpha=alpha, out=out)


def proj_dx(dy: torch.Tensor, weight: torch.Tensor) -> torch.Tensor:
    """Input gradient ``dy · weight`` of ``F.linear`` for 2-D ``dy`` (M, N_out) -> (M, N_in)."""
    if _proj_ok(dy, weight):
        return _ext.ops().proj(dy, weight, None, True, None, _force(), 1.0)
    if _f32_ok(dy, weight):
        dy, w = dy.contiguous(), weight.contiguous()
        M, K, N = dy.shape[0], dy.shape[1], w.shape[1]
        out = torch.empty(M, N, dtype=dy.dtype, device=dy.device)
        strided_gemm(dy, w, out, M=M, N=N, K=K, lda=K, ldb=N, ldc=N, b_mc=True, split_ok=False)
        return out
    return dy @ weight


def native_wgrad(dy: torch.Tensor, x: torch.Tensor) -> bool:
    """True when :func:`weight_grad` runs on the xdot MFMA kernels (16-bit GPU operands), False
    when it falls back to a library GEMM.

    Only the native path may run on a second stream beside other GEMMs: a library GEMM may pick
    a stream-K kernel whose workgroups spin on partial-tile flags and assume the grid is
    co-resident, and two such kernels in flight on two streams can hold every CU slot while
    waiting for each other's unscheduled producers (the fp32 module step stalled this way with
    the output-projection dW and dx GEMMs on two streams)."""
    return _ext.use_hip(dy, x) and dy.dtype == x.dtype and dy.dtype in (torch.bfloat16, torch.float16)


def weight_grad(dy: torch.Tensor, x: torch.Tensor, out_dtype: Optional[torch.dtype] = None) -> torch.Tensor:
    """``dyᵀ·x`` for 2-D ``dy`` (K, M) and ``x`` (K, N) -> (M, N), fp32 accumulation."""
    K, M = dy.shape
    N = x.shape[1]
    out_dtype = out_dtype or dy.dtype
    if _f32_ok(dy, x) and out_dtype == torch.float32:
        # exact fp32 on csrc/gemm_f32.hip; the long K (= rows) runs as K slabs + one ordered sum
        dy, x = dy.contiguous(), x.contiguous()
        out = torch.empty(M, N, dtype=torch.float32, device=dy.device)
        strided_gemm(dy, x, out, M=M, N=N, K=K, lda=M, ldb=N, ldc=N, a_mc=True, b_mc=True, split_ok=False)
        return out
    if not native_wgrad(dy, x):
        ct = torch.float32 if dy.dtype in (torch.bfloat16, torch.float16) else torch.promote_types(dy.dtype, x.dtype)
        return (dy.to(ct).t() @ x.to(ct)).to(out_dtype)
    dy = dy.contiguous()
    x = x.contiguous()
    if M % 128 == 0 and N % 128 == 0 and FLAGS.wgrad_kernel:
        # csrc/gemm_wgrad.hip: 128x128 tiles x K slabs (~2 workgroups per CU), fp32 partials, one
        # ordered sum (profiles/r4_s2.md)
        out = _ext.ops().wgrad(dy, x, out_dtype, 0)
        if out is not None:
            return out
    # 256x256 kernel.  K slabs of the 128x128 kernel are faster in isolation at short K (K = 3125:
    # 36 vs 44 µs at 768²) but not inside the step (emulated N=8 rank 1.350 vs 1.343 ms):
    # profiles/r2_wgrad_route.md; the slab path serves the shapes the 256x256 kernel does not take.
    if M % 8 == 0 and N % 8 == 0 and min(M, N) >= 128:
        # 256x256 LDS-DMA kernel: it picks the K split itself (fp32 slices, one vectorised
        # in-order reduction that also casts to the parameter dtype)
        out = torch.empty(M, N, dtype=out_dtype, device=dy.device)
        strided_gemm(dy, x, out, M=M, N=N, K=K, lda=M, ldb=N, ldc=N, a_mc=True, b_mc=True, path=_WGRAD_PATH)
        return out
    S = _splits(M, N, K)
    slab = K // S
    part = torch.empty(S + (1 if K % S else 0), M, N, dtype=torch.float32, device=dy.device)
    if slab > 0:
        strided_gemm(dy, x, part, M=M, N=N, K=slab, nb2=S, lda=M, ldb=N, ldc=N,
                     sA2=slab * M, sB2=slab * N, sC2=M * N, a_mc=True, b_mc=True)
    if K % S:
        r0 = S * slab
        strided_gemm(dy[r0:], x[r0:], part[S], M=M, N=N, K=K - r0, lda=M, ldb=N, ldc=N,
                     a_mc=True, b_mc=True)
    if (M * N) % 4 == 0:
        return _ext.ops().sum_partials(part, out_dtype)
    return part.sum(0).to(out_dtype)


def weight_grad_pair(dy0: torch.Tensor, x0: torch.Tensor, dy1: torch.Tensor, x1: torch.Tensor,
                     out_dtype: Optional[torch.dtype] = None):
    """``(dy0ᵀ·x0, dy1ᵀ·x1)``: both products in ONE launch of csrc/gemm_wgrad.hip where it takes
    them (their workgroups share the GPU instead of two under-filled launches back to back), else
    two :func:`weight_grad` calls."""
    dy0, x0 = dy0.reshape(-1, dy0.shape[-1]), x0.reshape(-1, x0.shape[-1])
    dy1, x1 = dy1.reshape(-1, dy1.shape[-1]), x1.reshape(-1, x1.shape[-1])
    out_dtype = out_dtype or dy0.dtype
    if (FLAGS.wgrad_kernel and FLAGS.wgrad_pair and native_wgrad(dy0, x0) and native_wgrad(dy1, x1)
            and dy0.dtype == dy1.dtype
            and all(t.shape[1] % 128 == 0 for t in (dy0, x0, dy1, x1))):
        outs = _ext.ops().wgrad2(dy0.contiguous(), x0.contiguous(), dy1.contiguous(), x1.contiguous(), out_dtype)
        if len(outs) == 2:
            return outs[0], outs[1]
    return weight_grad(dy0, x0, out_dtype), weight_grad(dy1, x1, out_dtype)


def linear_backward(dy: torch.Tensor, x: torch.Tensor, weight: torch.Tensor, need_dx: bool, need_dw: bool,
                    need_db: bool, join: bool = True, dw_dtype: Optional[torch.dtype] = None):
    """Gradients of ``F.linear(x, weight, bias)``: (dx, dw, db), each None when not needed.  dw is
    the split-K MFMA weight gradient (fp32 accumulation), in ``dw_dtype`` (default: the weight's;
    fp32 for GradSync's fp32 wire, :meth:`xdot.parallel.GradSync.wire_dtype`), db likewise.  When
    ``dy._xdot_ready_on`` names a stream, dw / db are computed there; ``join=False`` leaves ordering
    the current stream after them (and ``record_stream`` of dw / db on it) to the caller."""
    dx = dw = db = None
    dy2 = dy.reshape(-1, dy.shape[-1])
    if need_dx:
        dx = proj_dx(dy2, weight).view(*dy.shape[:-1], weight.shape[1])
    side = getattr(dy, "_xdot_ready_on", None)  # dy is complete on this stream (see below)
    if side is not None and need_dw and not native_wgrad(dy, x):
        side = None  # a library GEMM stays on the current stream (native_wgrad)
    cur = torch.cuda.current_stream(dy.device) if side is not None else None
    with torch.cuda.stream(side) if side is not None else contextlib.nullcontext():
        if need_dw:
            dw = weight_grad(dy2, x.reshape(-1, x.shape[-1]), dw_dtype or weight.dtype)
        if need_db:
            ct = torch.float32 if dy.dtype in (torch.bfloat16, torch.float16) else dy.dtype
            db = dy2.sum(0, dtype=ct).to(dw_dtype or dy.dtype)
    if side is not None and (need_dw or need_db):
        # the fused attention backward produced dy on its priority stream while its row-side
        # kernel still runs on `cur`: the weight / bias gradients run there too, overlapping
        # that kernel, and `cur` is ordered after them before they are handed on
        x.record_stream(side)
        dy.record_stream(side)
        if join:
            for t in (dw, db):
                if t is not None:
                    t.record_stream(cur)
            cur.wait_stream(side)
    return dx, dw, db


class LinearFn(torch.autograd.Function):
    @staticmethod
    @_ext.pinned
    def forward(ctx, x, weight, bias):
        ctx.save_for_backward(x, weight)
        ctx.has_bias = bias is not None
        return proj(x, weight, bias)

    @staticmethod
    @_ext.pinned
    def backward(ctx, dy):
        x, weight = ctx.saved_tensors
        return linear_backward(dy, x, weight, ctx.needs_input_grad[0], ctx.needs_input_grad[1],
                               ctx.has_bias and ctx.needs_input_grad[2])


def linear(x: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``F.linear`` on the projection GEMM with the split-K MFMA weight gradient for bf16/fp16 GPU
    tensors."""
    if x.is_cuda and x.dtype == weight.dtype and (x.dtype in (torch.bfloat16, torch.float16) or _f32_ok(x, weight)) \
            and _ext.use_hip(x):
        if torch.is_grad_enabled():
            return LinearFn.apply(x, weight, bias)
        return proj(x, weight, bias)
    return F.linear(x, weight, bias)
