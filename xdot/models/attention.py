"""``DistributedDotProductAttn`` — multi-head attention over time-sharded sequences.

Same constructor, forward signature, math and submodule names as the reference
(``distributed_dot_product/module.py:22-76``), so ``state_dict``s interchange:
``keys``/``queries``/``values``/``composition`` Linears, ``S = K·Qᵀ/√(key_dim/H)`` where
**``keys`` is the local/row side and ``queries`` the gathered side**, ``S[mask] = -inf``,
``P = softmax(S)``, ``O = P·V``, ``out = composition(merge(O))``.

Three execution paths, chosen by ``impl``:

``'materialized'`` — the reference's structure, op for op: ``RightTransposeMultiplication``
    → fused scale+mask+softmax kernel → ``FullMultiplication``.  Scores (B, H, T/N, T) are
    materialised once (bf16 on MI355X: 1.25 GB/rank at T=25000, N=8).
``'flash'`` — sequence-parallel fused attention (:mod:`xdot.parallel.attention`): K/V-side
    all-gather once, MFMA flash-attention kernels with online softmax (scores never exist in
    HBM), backward by recomputation with reduce-scatter of the gathered-side gradients.
    Required for long context (T=200000: materialised bf16 scores would be 80 GB per rank).
``'ring'`` — the same kernels fed by a ring of point-to-point RCCL hops
    (:mod:`xdot.parallel.ring`): the gathered side travels one rank-block at a time and is
    never resident in full; its gradient accumulator rides the ring back (no reduce-scatter).
``'auto'`` (default) — ``'flash'`` for bf16/fp16 GPU tensors with a supported head dim, else
    ``'materialized'``.

Extensions over the reference (all backward compatible): ``attn_mask=None`` means no mask,
``value_dim`` may differ from ``key_dim`` with several heads (the reference raises), any
float dtype works, and ``distributed=False`` gives the single-device ground truth.

Keyword-only knobs (each mirrors an environment flag, the argument wins):

``impl``        ``'auto'`` | ``'flash'`` | ``'ring'`` | ``'materialized'`` (above);
``fused``       ``True`` = ``impl='flash'``, ``False`` = ``impl='materialized'`` (SURVEY name);
``backend``     ``'auto'`` | ``'hip'`` | ``'torch'``: compute backend of this module's ops, forward
                and backward (``XDOT_BACKEND``); ``'torch'`` runs the torch reference math on GPU;
``dtype``       compute-dtype policy: e.g. ``torch.bfloat16`` runs projections and attention in
                bf16 while parameters / inputs stay fp32 (master weights); output in the input
                dtype.  ``None``: compute in the input dtype;
``chunk_plan``  row chunks of the fused path's all-gather / reduce-scatter pipeline
                (``XDOT_GATHER_CHUNKS``); the materialised path's chunking is ``offset``;
``comm``        communicator (default: the process group of :func:`xdot.init`).
"""
from __future__ import annotations

import math
from typing import Optional

import torch
import torch.nn as nn
from torch import Tensor

from .. import _ext
from ..ops.linear import linear
from ..ops.softmax import scale_mask_softmax
from ..parallel.autograd import FullMultiplication, RightTransposeMultiplication
from ..utils import comm as _comm
from ..utils.env import FLAGS

__all__ = ["DistributedDotProductAttn"]


def _adjacent(a: Tensor, b: Tensor) -> bool:
    return (a.is_contiguous() and b.is_contiguous() and a.dtype == b.dtype and a.device == b.device
            and tuple(a.shape[1:]) == tuple(b.shape[1:])
            and a.untyped_storage().data_ptr() == b.untyped_storage().data_ptr()
            and b.storage_offset() == a.storage_offset() + a.numel())


class _RowsView(torch.autograd.Function):
    """``cat([a, b], 0)`` as a no-copy view of the storage ``a`` and ``b`` share (``b`` stored
    right after ``a``); the gradient splits back into two row views."""

    @staticmethod
    def forward(ctx, a, b):
        ctx.n = a.shape[0]
        return a.detach().as_strided((a.shape[0] + b.shape[0],) + tuple(a.shape[1:]), a.stride(),
                                     a.storage_offset())

    @staticmethod
    def backward(ctx, g):
        return g[:ctx.n], g[ctx.n:]


def _stacked_rows(a: Tensor, b: Tensor) -> Tensor:
    """``cat([a, b], 0)`` for two parameters.  First use (or after ``.to()`` gave them separate
    storages): both are moved into ONE contiguous buffer (``.data`` rebound: the Parameter
    objects, their optimizer state and ``state_dict`` keys are unchanged); every later call is a
    view of it."""
    if not _adjacent(a, b):
        if not (isinstance(a, nn.Parameter) and isinstance(b, nn.Parameter) and a.dtype == b.dtype
                and a.device == b.device and tuple(a.shape[1:]) == tuple(b.shape[1:])) \
                or torch.is_inference_mode_enabled():
            # (under inference mode the packed buffer would be an inference tensor that later
            # in-place optimizer updates could not touch: no repack there)
            return torch.cat([a, b], 0)
        with torch.no_grad():
            packed = torch.empty((a.shape[0] + b.shape[0],) + tuple(a.shape[1:]), dtype=a.dtype, device=a.device)
            packed[:a.shape[0]].copy_(a)
            packed[a.shape[0]:].copy_(b)
            a.data = packed[:a.shape[0]]
            b.data = packed[a.shape[0]:]
    return _RowsView.apply(a, b)


class DistributedDotProductAttn(nn.Module):
    def __init__(self, key_dim: int, value_dim: Optional[int] = None, query_dim: Optional[int] = None,
                 num_heads: int = 1, add_bias: bool = False, offset: Optional[int] = 32,
                 distributed: bool = True, *, impl: str = "auto", fused: Optional[bool] = None,
                 backend: str = "auto", dtype: Optional[torch.dtype] = None, chunk_plan: Optional[int] = None,
                 comm: Optional[_comm.Communicator] = None):
        super().__init__()
        if fused is not None:
            if impl not in ("auto", "flash" if fused else "materialized"):
                raise ValueError(f"fused={fused} contradicts impl={impl!r}")
            impl = "flash" if fused else "materialized"
        if backend not in ("auto", "hip", "torch"):
            raise ValueError(f"backend must be auto|hip|torch, got {backend!r}")
        if dtype is not None and not (isinstance(dtype, torch.dtype) and dtype.is_floating_point):
            raise ValueError(f"dtype must be a floating torch.dtype or None, got {dtype!r}")
        if chunk_plan is not None and int(chunk_plan) < 1:
            raise ValueError(f"chunk_plan must be a positive number of row chunks, got {chunk_plan!r}")
        if key_dim % num_heads != 0:
            raise ValueError(f"key_dim {key_dim} not divisible by num_heads {num_heads}")
        value_dim = value_dim if value_dim is not None else key_dim
        query_dim = query_dim if query_dim is not None else key_dim
        if value_dim % num_heads != 0:
            raise ValueError(f"value_dim {value_dim} not divisible by num_heads {num_heads}")
        if impl not in ("auto", "flash", "materialized", "ring"):
            raise ValueError(f"impl must be auto|flash|materialized|ring, got {impl!r}")
        self.num_heads = num_heads
        self.value_dim = value_dim
        self.offset = offset
        self.distributed = distributed
        self.dim = key_dim // num_heads
        self.impl = impl
        self.backend = backend
        self.compute_dtype = dtype
        self.chunk_plan = None if chunk_plan is None else int(chunk_plan)
        self.comm = comm
        self.keys = nn.Linear(key_dim, key_dim, bias=add_bias)
        self.queries = nn.Linear(query_dim, key_dim, bias=add_bias)
        self.values = nn.Linear(value_dim, value_dim, bias=add_bias)
        self.composition = nn.Linear(value_dim, value_dim, bias=add_bias)
        # weakref to an attached xdot.parallel.GradSync (set by it): the fused node hands it the
        # parameter gradients as they are computed (early all-reduce)
        self._xdot_grad_sync = None

    # ------------------------------------------------------------------------------------
    def _pick_impl(self, x: Tensor) -> str:
        if self.impl != "auto":
            return self.impl
        from ..parallel import attention as pa

        with _ext.backend(self.backend):
            if self.compute_dtype is not None:
                x = x.to(self.compute_dtype) if x.is_floating_point() else x
            return "flash" if pa.flash_supported(x, self.dim, self.value_dim // self.num_heads) else "materialized"

    def forward(self, keys: Tensor, queries: Tensor, values: Tensor, attn_mask: Optional[Tensor] = None) -> Tensor:
        with _ext.backend(self.backend):
            cdt = self.compute_dtype
            if cdt is None or keys.dtype == cdt:
                return self._forward(keys, queries, values, attn_mask)
            out_dt = keys.dtype
            same_qv = queries is values
            keys_c = keys.to(cdt)
            queries_c = keys_c if queries is keys else queries.to(cdt)
            values_c = queries_c if same_qv else (keys_c if values is keys else values.to(cdt))
            return self._forward(keys_c, queries_c, values_c, attn_mask).to(out_dt)

    def _w(self, t: Optional[Tensor]) -> Optional[Tensor]:
        """A parameter in the compute dtype (autograd flows back to the master copy)."""
        if t is None or self.compute_dtype is None or t.dtype == self.compute_dtype:
            return t
        return t.to(self.compute_dtype)

    def _forward(self, keys: Tensor, queries: Tensor, values: Tensor, attn_mask: Optional[Tensor]) -> Tensor:
        scale = 1.0 / math.sqrt(self.dim)
        if self._pick_impl(keys) == "flash":
            from ..parallel import attention as pa
            from ..parallel.attention import seq_parallel_attention_packed, start_gather

            comm = (self.comm or _comm.get_comm()) if self.distributed else _comm.LocalComm()
            H, dk, dv = self.num_heads, self.dim, self.value_dim // self.num_heads
            Dp = pa.flash_head_dim(dk, dv) if keys.is_cuda else dk
            if keys.is_cuda and Dp is not None and (Dp != dk or Dp != dv):
                # head dims the kernels do not take (or value width != key width): every head
                # zero-padded to the next kernel dim, same scale 1/sqrt(dk)
                qv = self._project_qv(queries, values)
                qv = torch.cat([pa.pad_heads(qv[..., :H * dk], H, dk, Dp), pa.pad_heads(qv[..., H * dk:], H, dv, Dp)],
                               dim=-1)
                k = pa.pad_heads(self._proj(self.keys, keys), H, dk, Dp)
                o = seq_parallel_attention_packed(k, qv, attn_mask, H, scale, comm=comm)
                return self._proj(self.composition, pa.unpad_heads(o, H, dv, Dp))
            if attn_mask is not None and attn_mask.is_cuda and attn_mask.dim() == 3 and FLAGS.mask_async:
                # pack the mask on a side stream while the projection GEMMs run
                from ..ops import flash

                attn_mask = flash.prepare_mask_async(attn_mask.to(torch.bool), attn_mask.shape[0],
                                                     attn_mask.shape[1], attn_mask.shape[2])
            if (FLAGS.fused_module and queries is values and self.queries.in_features == self.values.in_features
                    and (self.compute_dtype is None or self.keys.weight.dtype == self.compute_dtype)):
                # the whole module as ONE autograd node (xdot.models.fused): same kernels, streams
                # and numerics, a fraction of the per-op host work
                from .fused import AttnBlockFn

                wq, wv = self.queries.weight, self.values.weight
                bq, bv = self.queries.bias, self.values.bias
                if isinstance(wq, nn.Parameter) and isinstance(wv, nn.Parameter):
                    _stacked_rows(wq, wv)  # (re)pack the two parameters into one storage once
                    if bq is not None:
                        _stacked_rows(bq, bv)
                gs = self._xdot_grad_sync() if self._xdot_grad_sync is not None else None
                sync = None
                if gs is not None and torch.is_grad_enabled():
                    gs.note_use(id(self))
                    sync = (gs, id(self))
                return AttnBlockFn.apply(keys, queries, attn_mask, self.keys.weight, self.keys.bias, wq, bq, wv, bv,
                                         self.composition.weight, self.composition.bias, self.num_heads, scale, comm,
                                         self.chunk_plan, sync, torch.is_grad_enabled())
            # gathered side first: its all-gather runs while the row-side GEMM computes
            qv = self._project_qv(queries, values)
            pending = start_gather(qv, comm, chunks=self.chunk_plan)
            k = self._proj(self.keys, keys)
            o = seq_parallel_attention_packed(k, qv, attn_mask, self.num_heads, scale, comm=comm, pending=pending)
            return self._proj(self.composition, o)
        if self._pick_impl(keys) == "ring":
            from ..parallel.ring import ring_attention_packed

            comm = (self.comm or _comm.get_comm()) if self.distributed else _comm.LocalComm()
            qv = self._project_qv(queries, values)
            k = self._proj(self.keys, keys)
            o = ring_attention_packed(k, qv, attn_mask, self.num_heads, scale, comm=comm)
            return self._proj(self.composition, o)
        k = self._proj(self.keys, keys)
        q = self._proj(self.queries, queries)
        v = self._proj(self.values, values)
        return self._proj(self.composition, self._materialized(k, q, v, attn_mask, scale))

    def _proj(self, layer: nn.Linear, x: Tensor) -> Tensor:
        """``layer(x)`` (compute dtype) with the split-K MFMA weight gradient (:mod:`xdot.ops.linear`)."""
        return linear(x, self._w(layer.weight), self._w(layer.bias))

    def _project_qv(self, queries: Tensor, values: Tensor) -> Tensor:
        """[q | v] packed (B, R, 2C): ONE GEMM when ``queries is values`` (self-attention), so
        the gathered side travels in one all-gather and its grads in one reduce-scatter.  The
        ``queries`` / ``values`` parameters share one storage (re-packed once after a ``.to()``),
        so the packed weight is a view: no concatenation kernel and no autograd node per step."""
        if queries is values and self.queries.in_features == self.values.in_features:
            w = self._w(_stacked_rows(self.queries.weight, self.values.weight))
            b = None
            if self.queries.bias is not None:
                b = self._w(_stacked_rows(self.queries.bias, self.values.bias))
            return linear(queries, w, b)
        return torch.cat([self._proj(self.queries, queries), self._proj(self.values, values)], dim=-1)

    def _materialized(self, k, q, v, attn_mask, scale):
        H = self.num_heads
        B, R = k.shape[0], k.shape[1]
        if H > 1:
            k = k.view(B, R, H, self.dim).transpose(1, 2)
            q = q.view(B, q.shape[1], H, self.dim).transpose(1, 2)
            v = v.view(B, v.shape[1], H, self.value_dim // H).transpose(1, 2)
        if self.distributed:
            comm = self.comm or _comm.get_comm()
            s = RightTransposeMultiplication.apply(k, q, self.offset, comm)
        else:
            s = torch.matmul(k, q.transpose(-1, -2))
        p = scale_mask_softmax(s, attn_mask, scale)
        if self.distributed:
            o = FullMultiplication.apply(p, v, self.offset, comm)
        else:
            o = torch.matmul(p, v)
        if H > 1:
            o = o.transpose(1, 2).reshape(B, R, self.value_dim)
        return o

    def extra_repr(self) -> str:
        return (f"heads={self.num_heads}, head_dim={self.dim}, value_dim={self.value_dim}, "
                f"offset={self.offset}, distributed={self.distributed}, impl={self.impl}, backend={self.backend}, "
                f"dtype={self.compute_dtype}, chunk_plan={self.chunk_plan}")
