"""Sequence-parallel fused ("flash") attention — the MI355X fast path of the module.

The reference materialises the (B, H, T/N, T) score block per rank and runs six chunked
distributed products per fwd+bwd (2x nt, 2x all, 2x tn), re-gathering the
same K/V data in backward.  This path keeps the reference's sharding (rank r owns rows
[rR, (r+1)R) of every sequence tensor; ``keys`` is the row side, ``queries``/``values`` the
gathered side) and its exact math, but restructures the work for HBM3E + MFMA + xGMI:

forward
  1. all-gather the gathered-side projections ``q`` and ``v`` ONCE (two RCCL all-gathers on
     the collective stream, issued before any compute);
  2. one flash-attention kernel per rank: S = k·qᵀ·scale, boolean mask, online softmax,
     O = P·v, all in registers/LDS; writes O (B, R, H·dv) in the layout the output Linear
     reads and the per-row log-sum-exp.  Nothing of size R x T touches HBM;
backward (recompute, no stored probabilities)
  3. δ = rowsum(dO ⊙ O);
  4. row-side kernel: dk = Σ_t dS·q_t  (dS = P ⊙ (dP − δ), dP = dO·v_tᵀ);
  5. gathered-side kernel: dq_t = Σ_rows dSᵀ·k, dv_t = Σ_rows Pᵀ·dO for ALL T gathered rows,
     as fp32 partials laid out rank-major, then ONE reduce-scatter each — the ``tn`` pattern
     of the reference, but fused and without re-gathering anything.

The gathered q/v are reused from forward (saved, T x (dh+dv) per head: 77 MB bf16 at
T=25000) instead of the reference's second round of gathers.  A fully masked row yields NaN
like the reference.  CPU tensors (and GPU dtypes the kernels do not take) run the same
schedule with a torch reference implementation of steps 2-5.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch
from torch import Tensor

from .. import _ext
from ..utils import comm as _comm
from ..utils.checks import check_consistent
from ..utils.env import FLAGS

__all__ = ["seq_parallel_attention", "seq_parallel_attention_packed", "start_gather", "flash_supported",
           "SeqParallelAttention"]

FLASH_HEAD_DIMS = (32, 64, 96, 128)


def flash_supported(x: Tensor, head_dim: int, v_head_dim: int) -> bool:
    if not x.is_cuda or x.dtype not in (torch.bfloat16, torch.float16):
        return False
    if head_dim not in FLASH_HEAD_DIMS or v_head_dim != head_dim:
        return False
    return _ext.use_hip(x) and hasattr(_ext.ops(), "flash_fwd")


# ----------------------------------------------------------------------------------------
# gather helpers
# ----------------------------------------------------------------------------------------
def _gather_rows(comm, x: Tensor, async_op: bool = True):
    """(B, R, C) -> (N, B, R, C) rank-major (row t = j*R + i of batch b at [j, b, i])."""
    n = comm.world_size
    x = x.contiguous()
    if n == 1:
        return _comm.Handle(out=x.unsqueeze(0)) if async_op else x.unsqueeze(0)
    out = torch.empty((n,) + tuple(x.shape), dtype=x.dtype, device=x.device)
    h = comm.all_gather_into(out, x, async_op=async_op)
    return h if async_op else out


def _as_global(g: Tensor) -> Tensor:
    """(N, B, R, C) -> (B, T, C) view/copy for the torch reference path."""
    n, B, R, C = g.shape
    return g.permute(1, 0, 2, 3).reshape(B, n * R, C)


# ----------------------------------------------------------------------------------------
# torch reference implementation of the per-rank compute (CPU / fallback / testing)
# ----------------------------------------------------------------------------------------
def _cdt(x):
    return torch.float64 if x.dtype == torch.float64 else torch.float32


def _ref_fwd(k, qg, vg, mask, H, scale):
    cdt = _cdt(k)
    B, R, C = k.shape
    dh = C // H
    dv = vg.shape[-1] // H
    qa, va = _as_global(qg), _as_global(vg)
    T = qa.shape[1]
    kh = k.view(B, R, H, dh).transpose(1, 2).to(cdt)
    qh = qa.view(B, T, H, dh).transpose(1, 2).to(cdt)
    vh = va.view(B, T, H, dv).transpose(1, 2).to(cdt)
    s = torch.matmul(kh, qh.transpose(-1, -2)) * scale
    if mask is not None:
        s = s.masked_fill(mask.unsqueeze(1), -float("inf"))
    lse = torch.logsumexp(s, dim=-1)                      # (B, H, R)
    p = torch.exp(s - lse.unsqueeze(-1))
    o = torch.matmul(p, vh)                               # (B, H, R, dv)
    return o.transpose(1, 2).reshape(B, R, H * dv).to(k.dtype), lse


def _ref_bwd(do, k, qg, vg, o, lse, mask, H, scale):
    cdt = _cdt(k)
    B, R, C = k.shape
    dh = C // H
    dv = vg.shape[-1] // H
    n = qg.shape[0]
    qa, va = _as_global(qg), _as_global(vg)
    T = qa.shape[1]
    kh = k.view(B, R, H, dh).transpose(1, 2).to(cdt)
    qh = qa.view(B, T, H, dh).transpose(1, 2).to(cdt)
    vh = va.view(B, T, H, dv).transpose(1, 2).to(cdt)
    doh = do.view(B, R, H, dv).transpose(1, 2).to(cdt)
    oh = o.view(B, R, H, dv).transpose(1, 2).to(cdt)
    s = torch.matmul(kh, qh.transpose(-1, -2)) * scale
    if mask is not None:
        s = s.masked_fill(mask.unsqueeze(1), -float("inf"))
    p = torch.exp(s - lse.unsqueeze(-1))
    delta = (doh * oh).sum(-1, keepdim=True)
    dp = torch.matmul(doh, vh.transpose(-1, -2))
    ds = p * (dp - delta) * scale
    dk = torch.matmul(ds, qh)                                          # (B, H, R, dh)
    dq_all = torch.matmul(ds.transpose(-1, -2), kh)                    # (B, H, T, dh)
    dv_all = torch.matmul(p.transpose(-1, -2), doh)                    # (B, H, T, dv)
    dk = dk.transpose(1, 2).reshape(B, R, H * dh)

    def rank_major(x, d):  # (B, H, T, d) -> (N, B, R, H*d)
        return x.transpose(1, 2).reshape(B, n, R, H * d).permute(1, 0, 2, 3).contiguous()

    return dk, rank_major(dq_all, dh), rank_major(dv_all, dv)


_SIDE = {}


def _side_stream(dev: torch.device) -> "torch.cuda.Stream":
    """Per-device high-priority compute stream of the backward (created once)."""
    i = dev.index if dev.index is not None else torch.cuda.current_device()
    if i not in _SIDE:
        _SIDE[i] = torch.cuda.Stream(device=i, priority=-1)
    return _SIDE[i]


# ----------------------------------------------------------------------------------------
class SeqParallelAttention(torch.autograd.Function):
    """Fused seq-parallel attention on a PACKED gathered-side operand ``qv`` = [q | v]
    (B, R, 2C): one all-gather in forward, one reduce-scatter in backward."""

    @staticmethod
    def forward(ctx, k, qv, mask, H, scale, comm, pending=None):
        check_consistent(comm, "seq_parallel_attention", k, qv, H)
        C = k.shape[-1]
        pending = pending if pending is not None else _gather_rows(comm, qv)
        use_hip = _ext.use_hip(k) and k.dtype in (torch.bfloat16, torch.float16)
        if use_hip:
            from ..ops import flash

            # the mask is packed while the gather is in flight
            mk = flash.prepare_mask(mask, k.shape[0], k.shape[1], qv.shape[1] * comm.world_size) \
                if mask is not None else None
            qvg = flash.gathered_to_btc(pending.wait())          # (B, T, 2C), a view for B = 1
            qg, vg = qvg[..., :C], qvg[..., C:]
            o, lse = flash.fwd(k, qg, vg, mk, H, scale)
        else:
            mk = mask
            qvg = pending.wait()                                 # (N, B, R, 2C)
            o, lse = _ref_fwd(k, qvg[..., :C], qvg[..., C:], mask, H, scale)
        ctx.save_for_backward(k, qvg, o, lse)
        ctx.mk, ctx.H, ctx.scale, ctx.comm, ctx.use_hip = mk, H, scale, comm, use_hip
        return o

    @staticmethod
    def backward(ctx, do):
        k, qvg, o, lse = ctx.saved_tensors
        comm, H, scale = ctx.comm, ctx.H, ctx.scale
        n = comm.world_size
        C = k.shape[-1]
        do = do.contiguous()

        def reduce_async(parts):  # (N, B, R, 2C) rank-major partials
            if n == 1:
                return None, parts[0]
            out = torch.empty(parts.shape[1:], dtype=parts.dtype, device=parts.device)
            return comm.reduce_scatter(out, parts, async_op=True), out

        if ctx.use_hip:
            from ..ops import flash

            qg, vg = qvg[..., :C], qvg[..., C:]
            # δ, then two independent kernels on two streams: 1) gathered-side grads for all T
            # columns on a HIGH-priority stream, followed there by 2) the ONE reduce-scatter,
            # and 3) the row-side dk on the current stream.  3) fills the partly occupied last
            # workgroup rounds of 1) while the priority keeps 1) (and so the start of the
            # collective) nearly as early as when it runs alone; 2) overlaps the rest of 3).
            # δ runs on the priority stream too, so 1) is queued right behind it while 3)
            # waits for δ: the column kernel reaches the GPU first and keeps the lead
            cur = torch.cuda.current_stream(do.device)
            hi = _side_stream(do.device)
            hi.wait_stream(cur)
            with torch.cuda.stream(hi):
                delta = flash.bwd_delta(do, o, H)
                ev = torch.cuda.Event()
                ev.record(hi)
                # partials rounded once to the compute dtype in the kernel (XDOT_GRAD_FP32=1
                # keeps fp32): half the epilogue stores and half the reduce-scatter bytes
                dkv, _ = flash.bwd_cols(do, k, qg, vg, o, lse, ctx.mk, H, scale, delta, fp32_out=FLAGS.grad_fp32)
                h, dqv = reduce_async(flash.btc_to_rank_major(dkv, n))
            cur.wait_event(ev)
            delta.record_stream(cur)
            dk = flash.bwd_rows(do, k, qg, vg, lse, delta, ctx.mk, H, scale)
            cur.wait_stream(hi)
            dqv.record_stream(cur)
        else:
            dk, dq_parts, dv_parts = _ref_bwd(do, k, qvg[..., :C], qvg[..., C:], o, lse, ctx.mk, H, scale)
            h, dqv = reduce_async(torch.cat([dq_parts, dv_parts], dim=-1))
        if h is not None:
            h.wait()
        return dk.to(k.dtype), dqv.to(k.dtype), None, None, None, None, None


def start_gather(qv: Tensor, comm: Optional[_comm.Communicator] = None) -> _comm.Handle:
    """Issue the all-gather of the packed gathered side early (e.g. before the row-side
    projection GEMM) and hand the handle to :func:`seq_parallel_attention_packed`."""
    comm = comm or _comm.get_comm()
    return _gather_rows(comm, qv.detach())


def seq_parallel_attention_packed(k: Tensor, qv: Tensor, mask: Optional[Tensor], num_heads: int, scale: float,
                                  comm: Optional[_comm.Communicator] = None,
                                  pending: Optional[_comm.Handle] = None) -> Tensor:
    """Fused sequence-parallel attention with a packed gathered side ``qv = [q | v]`` (B, R, 2C).

    ``pending``: the handle of :func:`start_gather` on this ``qv`` (the gather is issued here
    otherwise)."""
    comm = comm or _comm.get_comm()
    if k.dim() != 3 or qv.dim() != 3 or qv.shape[-1] <= k.shape[-1]:
        raise ValueError("seq_parallel_attention_packed expects k (B, R, C) and qv (B, R, C + Cv)")
    if mask is not None:
        T = qv.shape[1] * comm.world_size
        if tuple(mask.shape) != (k.shape[0], k.shape[1], T):
            raise ValueError(f"mask must be (B, R, T)=({k.shape[0]}, {k.shape[1]}, {T}), got {tuple(mask.shape)}")
        mask = mask.to(torch.bool)
    return SeqParallelAttention.apply(k, qv, mask, num_heads, float(scale), comm, pending)


def seq_parallel_attention(k: Tensor, q: Tensor, v: Tensor, mask: Optional[Tensor], num_heads: int,
                           scale: float, comm: Optional[_comm.Communicator] = None) -> Tensor:
    """Fused sequence-parallel attention on projected, head-interleaved (B, R, H*d) tensors.

    ``k``: row side (local rows), ``q``/``v``: gathered side (local shards), ``mask``: bool
    (B, R, T) with True = masked, or None.  Returns (B, R, H*dv) in ``k``'s dtype.
    """
    if k.dim() != 3 or q.dim() != 3 or v.dim() != 3:
        raise ValueError("seq_parallel_attention expects (B, R, H*d) tensors")
    return seq_parallel_attention_packed(k, torch.cat([q, v], dim=-1), mask, num_heads, scale, comm)
