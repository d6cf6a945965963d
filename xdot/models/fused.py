"""The whole module on the fused (flash) path as ONE autograd node.

Reference structure (``distributed_dot_product/module.py:41-76``): three input projections,
``RightTransposeMultiplication`` -> scale / mask / softmax -> ``FullMultiplication``, the
output projection -- each an autograd node whose backward the engine schedules separately
(``multiplication/ops.py:29-37, :49-54``).  On the flash path the per-node host work (Python
``Function.apply`` / ``backward`` dispatch, argument flattening, saved-tensor bookkeeping) is a
large share of the per-rank step's host time at N=8 (``profiles/r3_rank_host.md``), where the
GPU step is only ~1.4 ms.  :class:`AttnBlockFn` runs

    forward   [q|v] = x_qv Wqvᵀ (+b)  ->  all-gather issued  ->  k = x_k Wkᵀ (+b)
              ->  seq-parallel flash attention  ->  out = o Wcᵀ (+b)
    backward  do = dout Wc  ->  attention backward (both kernels, reduce-scatter)
              ->  dx_k  ->  dx_qv
              beside it: dWc / dbc on a second stream, under the attention backward; dWk / dbk
              there too, under the input-gradient GEMMs; dW[q|v] on the attention backward's
              priority stream as soon as the reduce-scatter lands (under the row-side kernel)

with the same kernels, streams and numerics as the per-op graph (``XDOT_FUSED_MODULE=0``
restores it), and hands back the eight parameter gradients and the input gradients in one go.
"""
from __future__ import annotations

import torch

from .. import _ext
from ..ops.linear import linear_backward, native_wgrad, proj, weight_grad_pair
from ..utils.env import FLAGS
from ..parallel.attention import SeqParallelAttention, gather_plan, prescale_wanted, start_gather

_LOG2E = 1.4426950408889634  # as the kernels' scale * log2 e (csrc/flash_common.h, csrc/reduce.hip)

__all__ = ["AttnBlockFn"]


class _Ctx:
    """Stand-in ``ctx`` for calling :class:`SeqParallelAttention`'s forward / backward inline."""

    def save_for_backward(self, *ts):
        self._saved = ts

    @property
    def saved_tensors(self):
        return self._saved


def _rows(a, b):
    """``cat([a, b], 0)``: a view when ``b`` is stored right after ``a`` (the module keeps the
    ``queries`` / ``values`` parameters in one storage), else a copy."""
    from .attention import _adjacent

    if _adjacent(a, b):
        return a.detach().as_strided((a.shape[0] + b.shape[0],) + tuple(a.shape[1:]), a.stride(), a.storage_offset())
    return torch.cat([a, b], 0)


def _wgrad_stream(t):
    """Second compute stream for the weight gradients that only the optimizer needs (None on
    the CPU, under HIP-graph capture, with ``XDOT_WGRAD_SIDE=0`` and when the weight gradients
    are library GEMMs: ``xdot.ops.linear.native_wgrad``)."""
    if not (t.is_cuda and FLAGS.wgrad_side and native_wgrad(t, t)) or torch.cuda.is_current_stream_capturing():
        return None
    from ..parallel.attention import _side_stream

    return _side_stream(t.device, 0)


def _ready_on(t, side):
    """``side`` ordered after the current stream's work so far (``t`` is complete there)."""
    side.wait_stream(torch.cuda.current_stream(t.device))
    return side


class AttnBlockFn(torch.autograd.Function):
    @staticmethod
    @_ext.pinned
    def forward(ctx, xk, xqv, mask, wk, bk, wq, bq, wv, bv, wc, bc, H, scale, comm, chunk_plan, sync=None,
                grad_on=True):
        wqv = _rows(wq, wv)
        bqv = _rows(bq, bv) if bq is not None else None
        n = comm.world_size
        B, R = xqv.shape[0], xqv.shape[1]
        gbuf = None
        if n > 1 and comm.inplace_gather and xqv.is_cuda and \
                len(gather_plan((B, R), xqv, comm, chunk_plan)) == 1:
            # the projection writes this rank's block of the gather output directly: the
            # all-gather runs in place (no copy of the own block; RCCL: sendbuff = recvbuff +
            # rank block, the xGMI pull kernel skips its own-block copy)
            gbuf = torch.empty((n, B, R, wqv.shape[0]), dtype=xqv.dtype, device=xqv.device)
            qv = gbuf[comm.rank]
            proj(xqv, wqv, bqv, out=qv.view(-1, qv.shape[-1]))
        else:
            qv = proj(xqv, wqv, bqv)
        pending = start_gather(qv, comm, chunks=chunk_plan, out=gbuf)  # in flight under the row-side GEMM
        # the row side's pre-scale (scale * log2 e) folded into the k projection: one rounding, no
        # separate pass (the attention backward's dk is w.r.t. the unscaled k either way)
        pre = xk.shape[-1] == wk.shape[1] and prescale_wanted(qv[..., :wk.shape[0]], qv, H)
        k = proj(xk, wk, bk, alpha=scale * _LOG2E if pre else 1.0)
        actx = _Ctx()
        actx.needs_input_grad = (any(ctx.needs_input_grad),) * 2  # a backward can run (score buffers)
        o = SeqParallelAttention.forward(actx, k, qv, mask, H, scale, comm, pending, pre, grad_on)  # k_prescaled
        out = proj(o, wc, bc)
        ctx.actx = actx
        ctx.sync = sync  # (GradSync, module key) or None
        ctx.params = (wk, bk, wq, bq, wv, bv, wc, bc)
        ctx.nq = wq.shape[0]
        ctx.has_b = (bk is not None, bq is not None, bc is not None)
        # the attention's tensors go through save_for_backward too (version checks, and a graph
        # retained for a second backward keeps them)
        asaved, actx._saved = actx._saved, None
        ctx.save_for_backward(xk, xqv, wk, wqv, wc, o, *asaved)
        return out

    @staticmethod
    @_ext.pinned
    def backward(ctx, dout):
        xk, xqv, wk, wqv, wc, o, *asaved = ctx.saved_tensors
        ctx.actx._saved = tuple(asaved)
        ng = ctx.needs_input_grad
        hk, hq, hc = ctx.has_b
        dout = dout.contiguous()
        # output projection: d(o) for the attention on this stream; its weight / bias gradients
        # (only needed by the optimizer) on a second stream, under the attention backward
        wk_, bk_, wq_, bq_, wv_, bv_, wc_, bc_ = ctx.params
        sync = None
        if ctx.sync is not None:
            gs, key = ctx.sync
            # deliver only when this forward was the parameters' ONLY use since the last wait():
            # a module called twice has its gradients summed by autograd (AccumulateGrad) first
            sync = gs if gs.sole_use(key) else None
        # weight gradients handed to GradSync in its wire dtype (fp32 for a bf16 module reduced in
        # fp32: straight from the kernels' fp32 sums, no conversion pass before the all-reduce)
        wdt = (lambda *ps: torch.float32 if any(p is not None and sync.wire_dtype(p) == torch.float32 for p in ps)
               else None) if sync is not None else (lambda *ps: None)
        side = _wgrad_stream(dout)
        if side is None:
            do, dwc, dbc = linear_backward(dout, o, wc, True, ng[9], hc and ng[10], dw_dtype=wdt(wc_, bc_))
        else:
            do, _, _ = linear_backward(dout, o, wc, True, False, False)
            dout._xdot_ready_on = _ready_on(dout, side)
            _, dwc, dbc = linear_backward(dout, o, wc, False, ng[9], hc and ng[10], join=False, dw_dtype=wdt(wc_, bc_))
        # the current stream is only looked up when a side stream is in play (host cost per call)
        cur = torch.cuda.current_stream(dout.device) if side is not None else None
        if sync is not None:  # hand the output projection's gradients to GradSync now: their
            # all-reduce runs under the attention backward (stream None: the current one)
            sync.deliver([(wc_, dwc), (bc_, dbc)], stream=side)
            dwc = dbc = None
        dk, dqv = SeqParallelAttention.backward(ctx.actx, do)[:2]
        # the row-side weight gradient also runs beside the input-gradient GEMMs that follow
        # d[q|v] may be ready on the backward's priority stream (``_xdot_ready_on``): its weight
        # gradient runs there, under the row-side kernel (linear_backward)
        qv_on = getattr(dqv, "_xdot_ready_on", None) if native_wgrad(dqv, xqv) else None  # (as linear_backward)
        need_wk, need_wqv = ng[3], ng[5] or ng[7]
        kdt, qvdt = wdt(wk_, bk_), wdt(wq_, bq_, wv_, bv_)
        if side is None and qv_on is None and need_wk and need_wqv:
            # one stream: dWk and dW[q|v] in ONE launch (weight_grad_pair)
            dxk, _, dbk = linear_backward(dk, xk, wk, ng[0], False, hk and ng[4], dw_dtype=kdt)
            dxqv, _, dbqv = linear_backward(dqv, xqv, wqv, ng[1], False, hq and (ng[6] or ng[8]), dw_dtype=qvdt)
            dwk, dwqv = weight_grad_pair(dk, xk, dqv, xqv, kdt or qvdt or wk.dtype)
        else:
            if side is None:
                dxk, dwk, dbk = linear_backward(dk, xk, wk, ng[0], need_wk, hk and ng[4], dw_dtype=kdt)
            else:
                dk._xdot_ready_on = _ready_on(dk, side)
                dxk, _, _ = linear_backward(dk, xk, wk, ng[0], False, False)
                _, dwk, dbk = linear_backward(dk, xk, wk, False, need_wk, hk and ng[4], join=False, dw_dtype=kdt)
            dxqv, dwqv, dbqv = linear_backward(dqv, xqv, wqv, ng[1], need_wqv, hq and (ng[6] or ng[8]), dw_dtype=qvdt)
        n = ctx.nq
        dwq = dwv = dbq = dbv = None
        # the packed products cover both halves; hand back only what is asked for (a frozen
        # queries weight next to a trained values weight gets None, and is never delivered)
        if dwqv is not None:
            dwq, dwv = (dwqv[:n] if ng[5] else None), (dwqv[n:] if ng[7] else None)
        if dbqv is not None:
            dbq, dbv = (dbqv[:n] if ng[6] else None), (dbqv[n:] if ng[8] else None)
        if sync is not None:
            qv_pairs, k_pairs = [(wq_, dwq), (bq_, dbq), (wv_, dwv), (bv_, dbv)], [(wk_, dwk), (bk_, dbk)]
            if qv_on is side:  # one call: the buckets it completes share one grouped all-reduce
                sync.deliver(qv_pairs + k_pairs, stream=side)
            else:
                sync.deliver(qv_pairs, stream=qv_on)
                sync.deliver(k_pairs, stream=side)
            dwq = dbq = dwv = dbv = dwk = dbk = None
        if side is not None:  # the gradients handed on are complete on this stream
            cur.wait_stream(side)
            for t in (dwc, dbc, dwk, dbk) + tuple(p.grad for p in ctx.params if p is not None and sync is not None):
                if t is not None:
                    t.record_stream(cur)
        # the attention's tensors were only borrowed from ctx.saved_tensors (rebuilt from there by
        # every backward): do not keep them alive through the node after this backward
        ctx.actx._saved = None
        return (dxk, dxqv, None, dwk, dbk, dwq, dbq, dwv, dbv, dwc, dbc, None, None, None, None, None, None)
