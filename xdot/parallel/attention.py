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

from typing import List, Optional, Tuple

import torch
from torch import Tensor

from .. import _ext
from ..utils import comm as _comm
from ..utils.checks import check_consistent
from ..utils.env import FLAGS

__all__ = ["seq_parallel_attention", "seq_parallel_attention_packed", "start_gather", "flash_supported",
           "SeqParallelAttention"]

# D <= 128: the tuned families (csrc/flash_fwd.hip, flash_bwd.hip, flash_f32.hip); 160-384: the
# wide-head family (csrc/flash_wide.hip: the reference's example.py 768 / 2 heads = 384 and its
# num_heads = 1 gradient test at 256).  Exact fp32 heads past 256 need the score buffer.
FLASH_HEAD_DIMS = (32, 64, 96, 128, 160, 192, 256, 384)
WIDE_F32_NEEDS_SCORES = 256
# bf16/fp16: 32x32x16 MFMA kernels; fp32: exact-f32 MFMA kernels — the reference's own precision
# without materialised scores
FLASH_DTYPES = (torch.bfloat16, torch.float16, torch.float32)


def flash_head_dim(head_dim: int, v_head_dim: int) -> Optional[int]:
    """The kernel head dim a (key, value) head pair runs at: itself when both are equal and a
    kernel dim, else the smallest kernel dim holding both (heads zero-padded: zero key / query
    columns add nothing to a score, zero value columns give zero outputs that are dropped), or
    None past 384."""
    m = max(head_dim, v_head_dim)
    return next((d for d in FLASH_HEAD_DIMS if d >= m), None)


def pad_heads(x: Tensor, H: int, d: int, Dp: int) -> Tensor:
    """(B, R, H*d) -> (B, R, H*Dp), every head zero-padded from d to Dp columns (differentiable)."""
    if d == Dp:
        return x
    B, R = x.shape[0], x.shape[1]
    return torch.nn.functional.pad(x.reshape(B, R, H, d), (0, Dp - d)).reshape(B, R, H * Dp)


def unpad_heads(x: Tensor, H: int, d: int, Dp: int) -> Tensor:
    """(B, R, H*Dp) -> (B, R, H*d): the first d columns of every head."""
    if d == Dp:
        return x
    B, R = x.shape[0], x.shape[1]
    return x.reshape(B, R, H, Dp)[..., :d].reshape(B, R, H * d)


def flash_supported(x: Tensor, head_dim: int, v_head_dim: int) -> bool:
    """The flash kernels take this (dtype, device, head dims), directly or zero-padded
    (:func:`flash_head_dim`)."""
    if not x.is_cuda or x.dtype not in FLASH_DTYPES:
        return False
    if flash_head_dim(head_dim, v_head_dim) is None:
        return False
    return _ext.use_hip(x) and hasattr(_ext.ops(), "flash_fwd")


def _hip_ok(k: Tensor, qv: Tensor, H: int) -> bool:
    """The HIP kernels take this call: a GPU bf16/fp16 row side, a supported head dim and a
    value width equal to the key width (otherwise the torch path runs, as documented)."""
    C = k.shape[-1]
    return (k.is_cuda and k.dtype in FLASH_DTYPES and C % H == 0
            and C // H in FLASH_HEAD_DIMS and qv.shape[-1] == 2 * C and _ext.use_hip(k)
            and hasattr(_ext.ops(), "flash_fwd"))


# ----------------------------------------------------------------------------------------
# gather helpers
# ----------------------------------------------------------------------------------------
def _gather_rows(comm, x: Tensor, async_op: bool = True, out: Optional[Tensor] = None):
    """(B, R, C) -> (N, B, R, C) rank-major (row t = j*R + i of batch b at [j, b, i]).  ``out``:
    the (N, B, R, C) output, whose block ``rank`` may already hold ``x`` (in-place gather)."""
    n = comm.world_size
    x = x.contiguous()
    if n == 1:
        return _comm.Handle(out=x.unsqueeze(0)) if async_op else x.unsqueeze(0)
    if out is None:
        out = torch.empty((n,) + tuple(x.shape), dtype=x.dtype, device=x.device)
    h = comm.all_gather_into(out, x, async_op=async_op)
    return h if async_op else out


def _row_chunks(n: int, R: int, hip: bool, nchunks: Optional[int] = None) -> List[Tuple[int, int]]:
    """Row chunks (r0, rc) of every rank's shard for the pipelined gather of the fused path:
    with several ranks the gathered side can travel in ``XDOT_GATHER_CHUNKS`` all-gathers so
    chunk c+1 is in flight while the kernels consume chunk c (and, in backward, chunk c's
    reduce-scatter runs while chunk c+1's gradients are computed).  Default (auto): 2 chunks
    from 8 ranks on, else 1 — measured on the emulated rank step with a 300 GB/s collective
    link model: N=8 1.621 -> 1.577 ms with 2 chunks, N=4 2.459 -> 2.471 ms (without any
    transfer time 2 chunks cost 23 / 55 µs of compute), profiles/r2_gather_chunks.md."""
    if n == 1:
        return [(0, R)]
    auto = 2 if n >= 8 else 1
    nc = nchunks or ((FLAGS.gather_chunks or auto) if hip else 1)
    nc = max(1, min(nc, R if nchunks else R // 64))  # an explicit plan is honoured down to 1-row chunks
    base, extra = divmod(R, nc)
    out, r0 = [], 0
    for c in range(nc):
        rc = base + (1 if c < extra else 0)
        out.append((r0, rc))
        r0 += rc
    return out


class _PendingGather:
    """All-gathers of the row chunks of one packed operand, issued back to back on the
    collective stream; ``wait(c)`` orders the current stream after chunk c only.

    With several chunks every chunk lands in its own slice of ONE buffer: chunk c's gather
    output (N, B, rc, ·) starts where chunk c-1's ends, so for B = 1 the buffer read as
    (1, T, ·) holds every gathered row in (chunk, source rank, row) order — a column
    permutation of the rank-major order that attention does not see (the mask columns are
    permuted to match, :func:`_perm_cols`), and the backward runs ONE kernel pair over it."""

    def __init__(self, comm, x: Tensor, chunks: List[Tuple[int, int]], out: Optional[Tensor] = None):
        self.chunks = chunks
        self.n = n = comm.world_size
        x = x.contiguous()
        self.flat = None
        if n > 1 and len(chunks) > 1:
            self.flat = torch.empty(n * x.numel(), dtype=x.dtype, device=x.device)
        self.handles = []
        off = 0
        for r0, rc in chunks:
            xc = x[:, r0:r0 + rc]
            if self.flat is None:
                self.handles.append(_gather_rows(comm, xc, out=out))
                continue
            out = self.flat[off:off + n * xc.numel()].view((n,) + tuple(xc.shape))
            off += out.numel()
            self.handles.append(comm.all_gather_into(out, xc.contiguous(), async_op=True))
        self._bufs: List[Optional[Tensor]] = [None] * len(chunks)

    def wait(self, c: int) -> Tensor:
        if self._bufs[c] is None:
            self._bufs[c] = self.handles[c].wait()          # (N, B, rc, 2C)
        return self._bufs[c]

    def wait_all(self) -> List[Tensor]:
        return [self.wait(c) for c in range(len(self.chunks))]

    def permuted(self) -> Optional[Tensor]:
        """(1, T, ·) view of the single buffer in (chunk, rank, row) column order (B = 1, several
        chunks, every chunk waited for), else None."""
        if self.flat is None or self._bufs[0].shape[1] != 1 or any(b is None for b in self._bufs):
            return None
        return self.flat.view(1, -1, self._bufs[0].shape[-1])


def _perm_cols(B: int, R: int, n: int, chunks: List[Tuple[int, int]]):
    """Mask columns in the (chunk, source rank, row) order of :meth:`_PendingGather.permuted`."""
    def view(m):
        m4 = m.reshape(B, R, n, R)
        return torch.cat([m4[..., r0:r0 + rc].reshape(B, R, n * rc) for r0, rc in chunks], dim=-1)
    return view


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


def _ref_fwd_partial(k, kc, vc, mask, H, scale):
    """One column segment of the forward in torch: ``kc``/``vc`` (B, Tseg, ·) in the segment's
    column order, ``mask`` (B, R, Tseg) or None -> (o (B, R, H*dv) normalised over the
    segment, lse (B, H, R)); a row the segment masks entirely gets o = 0, lse = -inf."""
    cdt = _cdt(k)
    B, R, C = k.shape
    dh = C // H
    T = kc.shape[1]
    dv = vc.shape[-1] // H
    kh = k.view(B, R, H, dh).transpose(1, 2).to(cdt)
    qh = kc.reshape(B, T, H, dh).transpose(1, 2).to(cdt)
    vh = vc.reshape(B, T, H, dv).transpose(1, 2).to(cdt)
    s = torch.matmul(kh, qh.transpose(-1, -2)) * scale
    if mask is not None:
        s = s.masked_fill(mask.unsqueeze(1), -float("inf"))
    lse = torch.logsumexp(s, dim=-1)
    p = torch.exp(s - lse.clamp_min(torch.finfo(cdt).min).unsqueeze(-1))
    o = torch.matmul(p, vh)
    return o.transpose(1, 2).reshape(B, R, H * dv), lse


def _ref_combine(parts, dtype):
    """Merge segment partials [(o, lse)] -> (o in ``dtype``, lse); NaN for fully masked rows."""
    L = torch.stack([l for _, l in parts])                      # (S, B, H, R)
    lse = torch.logsumexp(L, dim=0)
    w = torch.exp(L - lse.unsqueeze(0))                         # NaN only where every segment is -inf
    B, H, R = lse.shape
    o = sum(wi.transpose(1, 2).repeat_interleave(oi.shape[-1] // H, dim=-1) * oi
            for wi, (oi, _) in zip(w, parts))
    return o.to(dtype), lse


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


def _segment_plan(n: int, rank: int, nchunks: int, local_first: bool) -> List[Tuple[int, int, int]]:
    """Peer segments (chunk c, source ranks j0..j1-1) of the segmented forward, in launch order;
    the own rank is left out of every chunk when its block runs first."""
    plan = []
    for c in range(nchunks):
        ranges = [(0, rank), (rank + 1, n)] if local_first else [(0, n)]
        plan += [(c, j0, j1) for j0, j1 in ranges if j1 > j0]
    return plan


def _mask_cols(B: int, R: int, n: int, j0: int, j1: int, r0: int, rc: int):
    """Mask columns of source ranks j0..j1-1, rows r0..r0+rc of each (global column j*R + r0 + i)."""
    return lambda m: m.reshape(B, R, n, R)[..., j0:j1, r0:r0 + rc].reshape(B, R, (j1 - j0) * rc)


def _segmented_forward(k, qv, mask, H, scale, pending, n, rank, use_hip, prescaled, fp32_mode=0):
    """Forward of a multi-rank step as column segments merged by one log-sum-exp combine:
    the rank's OWN [q|v] block first (it needs no communication, so its partial runs while the
    all-gather is in flight), then each gathered chunk's peer blocks as soon as that chunk
    lands.  Every segment is a subset of a row's columns, so the partials (o normalised over
    the segment, its lse) merge exactly.  -> (o, lse, gathered buffers saved for backward)."""
    B, R, C = k.shape
    chunks = pending.chunks
    local_first = FLAGS.local_first
    plan = _segment_plan(n, rank, len(chunks), local_first)
    own = _mask_cols(B, R, n, rank, rank + 1, 0, R)
    if use_hip:
        from ..ops import flash

        ops = _ext.ops()
        if local_first and 0 < rank < n - 1 and SEGMENT_MERGE:
            # a middle rank's peers sit on both sides of its own block in every chunk: ONE partial
            # over the whole chunk with the own columns masked out (their tiles are skipped whole,
            # two boundary tiles per row block take the masked path) instead of two launches
            plan = [(c, 0, -1) for c in range(len(chunks))]
        widths = ([R] if local_first else []) + [(n if j1 == -1 else j1 - j0) * chunks[c][1] for c, j0, j1 in plan]
        ns = [int(ops.flash_splits(B, R, w, H, False)) for w in widths]
        opart = torch.empty(sum(ns), B, R, C, dtype=torch.float32, device=k.device)
        lpart = torch.empty(sum(ns), B, H, R, dtype=torch.float32, device=k.device)
        slot = [0, 0]  # next partial slot, next entry of ns

        def run(kc, vc, mk):
            bits, flags = (mk.bits, mk.flags) if mk is not None else (None, None)
            nsi = ns[slot[1]]
            ops.flash_fwd_partial(k, flash._kv(kc), flash._kv(vc), bits, flags, int(H), float(scale), opart, lpart,
                                  slot[0], nsi, prescaled, fp32_mode)
            slot[0] += nsi
            slot[1] += 1

        if local_first:
            mk = flash.prepare_mask_cached(mask, B, R, R, tag=("own", rank, n), view=own)
            run(qv[..., :C], qv[..., C:], mk)
        bufs = []
        for c, (r0, rc) in enumerate(chunks):
            g = flash.gathered_to_btc(pending.wait(c))          # (B, N*rc, 2C)
            bufs.append(g)
            for _, j0, j1 in (p for p in plan if p[0] == c):
                if j1 == -1:  # merged: every rank of the chunk, the own columns masked out
                    mk = _own_excluded_mask(mask, B, R, n, rank, r0, rc, k.device)
                    run(g[..., :C], g[..., C:], mk)
                    continue
                mk = flash.prepare_mask_cached(mask, B, R, (j1 - j0) * rc, tag=("seg", r0, rc, n, j0, j1),
                                               view=_mask_cols(B, R, n, j0, j1, r0, rc))
                seg = g[:, j0 * rc:j1 * rc]
                run(seg[..., :C], seg[..., C:], mk)
        o, lse = ops.flash_fwd_combine(opart, lpart, int(H), k)
        perm = pending.permuted()
        return o, lse, ([perm] if perm is not None else bufs)
    parts = []
    if local_first:
        parts.append(_ref_fwd_partial(k, qv[..., :C], qv[..., C:], None if mask is None else own(mask), H, scale))
    gs = []
    for c, (r0, rc) in enumerate(chunks):
        g = pending.wait(c)                                      # (N, B, rc, 2C)
        gs.append(g)
        for _, j0, j1 in (p for p in plan if p[0] == c):
            seg = _as_global(g[j0:j1])
            m = None if mask is None else _mask_cols(B, R, n, j0, j1, r0, rc)(mask)
            parts.append(_ref_fwd_partial(k, seg[..., :C], seg[..., C:], m, H, scale))
    o, lse = _ref_combine(parts, k.dtype)
    return o, lse, [torch.cat(gs, dim=2) if len(gs) > 1 else gs[0]]


_OWN_EX = {}
# False: a middle rank launches one partial per peer range (A/B diagnostics: bench_rank.py --no-seg-merge)
SEGMENT_MERGE = True


def _own_excluded_mask(mask, B: int, R: int, n: int, rank: int, r0: int, rc: int, dev):
    """Packed (B, R, n*rc) mask of one gather chunk with this rank's own columns masked (they
    ran first, under the all-gather), OR-ed with the user mask's columns of the chunk.  Cached:
    on the user mask (MASK_CACHE) or, without one, per shape."""
    from ..ops import flash

    def own_cols(m):
        m = m.clone()
        m[..., rank * rc:(rank + 1) * rc] = True
        return m

    if mask is not None:
        packed = flash.prepare_mask_cached(mask, B, R, n * rc, tag=("segx", r0, rc, n, rank),
                                           view=lambda m: own_cols(_mask_cols(B, R, n, 0, n, r0, rc)(m)))
        if packed is not None:
            return packed
    key = (B, R, n, rank, rc, dev)
    if key not in _OWN_EX:
        if len(_OWN_EX) >= 8:
            _OWN_EX.pop(next(iter(_OWN_EX)))
        _OWN_EX[key] = flash.prepare_mask(own_cols(torch.zeros(B, R, n * rc, dtype=torch.bool, device=dev)),
                                          B, R, n * rc)
    return _OWN_EX[key]


_SIDE = {}
# The fused backward runs its gathered-side half on a high-priority side stream so the row-side
# kernel fills the column kernel's last, mostly empty workgroup round.  Eager, on one MI355X
# (benchmarks/graph_ab.py, profiles/r3_graph.md), two streams vs one: N=1 8.18 vs 8.60 ms, N=2
# rank 4.38 vs 4.59, N=4 rank 2.40 vs 2.46, N=8 rank 1.39 vs 1.43 (an earlier box: 1.43 vs 1.40,
# within box noise).  Under HIP-graph capture the side stream's priority is lost and two streams
# replay 19-32 % slower at N=1/2, so a captured backward uses one stream.
# ONE_STREAM_BACKWARD: None = that rule, True / False = force (A/B diagnostics).
ONE_STREAM_BACKWARD = None


def _two_stream_backward(R: int) -> bool:
    if ONE_STREAM_BACKWARD is not None:
        return not ONE_STREAM_BACKWARD
    return not torch.cuda.is_current_stream_capturing()


def _side_stream(dev: torch.device, priority: int = -1, tag: str = "") -> "torch.cuda.Stream":
    """Per-device compute stream of the backward (created once per priority and tag; -1 = high)."""
    i = dev.index if dev.index is not None else torch.cuda.current_device()
    if (i, priority, tag) not in _SIDE:
        _SIDE[(i, priority, tag)] = torch.cuda.Stream(device=i, priority=priority)
    return _SIDE[(i, priority, tag)]


_EV = {}


def _prep_event(dev) -> "torch.cuda.Event":
    """One reusable event per device for "δ is ready" (a stream wait captures the event's state at
    the call, so re-recording it next step is safe): no event creation per backward."""
    i = dev.index if dev.index is not None else torch.cuda.current_device()
    if i not in _EV:
        _EV[i] = torch.cuda.Event()
    return _EV[i]


class _on_stream:
    """``with _on_stream(s, cur):`` makes ``s`` current and restores ``cur`` (the caller's
    current stream, already looked up).  Same effect as ``torch.cuda.stream(s)`` on one device
    without its device-index and current-stream lookups: 0.9 vs 5.8 µs of host per switch on
    MI355X (``benchmarks/micro/stream_ctx.py``)."""
    __slots__ = ("s", "cur")

    def __init__(self, s, cur):
        self.s, self.cur = s, cur

    def __enter__(self):
        if self.s is not self.cur:
            torch.cuda.set_stream(self.s)
        return self.s

    def __exit__(self, *exc):
        if self.s is not self.cur:
            torch.cuda.set_stream(self.cur)
        return False


def prescale_wanted(k_like: Tensor, qv_like: Tensor, H: int) -> bool:
    """The HIP path will run on pre-scaled rows for a row side shaped / typed like ``k_like``
    (the condition :meth:`SeqParallelAttention.forward` applies)."""
    return (_hip_ok(k_like, qv_like, H) and FLAGS.prescale and k_like.numel() % 8 == 0
            and k_like.dtype != torch.float32)


# ----------------------------------------------------------------------------------------
class SeqParallelAttention(torch.autograd.Function):
    """Fused seq-parallel attention on a PACKED gathered-side operand ``qv`` = [q | v]
    (B, R, 2C): all-gather(s) in forward, reduce-scatter(s) in backward.  With several ranks
    the gathered side moves in row chunks (:func:`_row_chunks`): the kernels run per chunk
    into split partials (merged by one combine) so communication overlaps compute."""

    @staticmethod
    @_ext.pinned
    def forward(ctx, k, qv, mask, H, scale, comm, pending=None, k_prescaled=False, grad_on=True):
        """``k_prescaled``: ``k`` already holds ``rows * scale * log2 e`` (:func:`prescale_wanted`;
        the fused module folds it into the k projection's epilogue).  ``grad_on``: grad mode at the
        call (inside ``forward`` it is always off, and ``needs_input_grad`` ignores it)."""
        check_consistent(comm, "seq_parallel_attention", k, qv, H)
        C = k.shape[-1]
        B, R = k.shape[0], k.shape[1]
        n, rank = comm.world_size, comm.rank
        use_hip = _hip_ok(k, qv, H)
        if pending is None:
            pending = _PendingGather(comm, qv, _row_chunks(n, qv.shape[1], use_hip))
        chunks = pending.chunks
        prescaled = False
        fm = 0  # fp32 kernel family (XDOT_FP32_MODE), fixed at forward for the backward too
        packed_full = None  # the whole-row packed mask, when the caller packed it ahead
        D = C // H
        if use_hip:
            from ..ops import flash

            fm = flash.fp32_code(k.dtype) if D <= 128 else 0  # wide fp32 heads are exact only
            # the row side pre-multiplied by scale*log2 e once (XDOT_PRESCALE, default on): the
            # forward and both backward kernels read this same buffer and seed their score
            # accumulators instead of scaling every score (saved in place of k for backward)
            prescaled = FLAGS.prescale and (k.numel() % 8 == 0) and k.dtype != torch.float32
            if prescaled and not k_prescaled:
                k = flash.prescale(k, scale)
            if isinstance(mask, flash.PendingMask):
                if len(chunks) == 1:
                    packed_full = mask.get()
                mask = mask.raw
        mask = getattr(mask, "raw", mask)
        segmented = n > 1 and (FLAGS.local_first or len(chunks) > 1)
        sbuf = dsbuf = None
        # a backward can run on this forward (grad mode is off inside Function.forward: autograd's
        # needs_input_grad, or the fused node's, says it); without one no score buffer is taken
        # (no 20 GB allocation and store pass for inference / no_grad forwards)
        need_bwd = bool(grad_on) and any(getattr(ctx, "needs_input_grad", (True,))[:2])
        if use_hip and k.dtype == torch.float32 and need_bwd and (len(chunks) == 1 or B == 1):
            # fp32 (exact or split): score buffer (flash.score_buffer) when it fits: the backward
            # then reads S / dS instead of recomputing them.  One kernel over the whole gathered
            # side (in fp32 the own-block-first segmentation hides < 5 % of a rank's forward)
            if flash.ds_only_wanted(fm, D):  # dS-only: nothing stored by the forward
                dsbuf = flash.ds_buffer(B, H, R, n * qv.shape[1], k.device)
                if dsbuf is not None:
                    segmented = False
            else:
                # the fused exact column pass overwrites S with dS in place: no second buffer
                sbs = flash.score_buffers(B, H, R, n * qv.shape[1], k.device,
                                          dsbuf=not flash.fused_cols_wanted(fm, D))
                if sbs is not None:
                    sbuf, dsbuf = sbs
                    segmented = False
        if use_hip and k.dtype == torch.float32 and D > WIDE_F32_NEEDS_SCORES and sbuf is None and need_bwd:
            # no kernel recomputes an fp32 head this wide (three D-wide register sets) and the torch
            # path would materialise a score matrix larger than the buffer that did not fit
            raise RuntimeError(
                f"xdot: training exact-fp32 attention at head dim {D} needs the flash score buffer "
                f"({4 * flash.score_buffer_numel(B, H, R, n * qv.shape[1]) / 2**30:.1f} GiB), which does not fit "
                f"within XDOT_FP32_SCORES_FRAC={FLAGS.fp32_scores_frac} of the free device memory: shorten the "
                "sequence, raise XDOT_FP32_SCORES_FRAC, or run the module in bf16")
        if not segmented:
            if use_hip:
                if len(chunks) > 1:  # several gather chunks, one buffer in (chunk, rank, row) order
                    pending.wait_all()
                    qvg = pending.permuted()
                    mk = flash.prepare_mask_cached(mask, B, R, n * R, tag=("perm", tuple(chunks), n),
                                                   view=_perm_cols(B, R, n, chunks))
                else:
                    mk = packed_full if packed_full is not None else flash.prepare_mask_cached(mask, B, R, n * R)
                    qvg = flash.gathered_to_btc(pending.wait(0))     # (B, T, 2C), a view for B = 1
                o, lse = flash.fwd(k, qvg[..., :C], qvg[..., C:], mk, H, scale, prescaled=prescaled, fp32_mode=fm,
                                   sbuf=sbuf)
                bufs, mks = [qvg], [mk]
            else:
                qvg = pending.wait(0)                            # (N, B, R, 2C)
                o, lse = _ref_fwd(k, qvg[..., :C], qvg[..., C:], mask, H, scale)
                bufs, mks = [qvg], [mask]
        else:
            o, lse, bufs = _segmented_forward(k, qv, mask, H, scale, pending, n, rank, use_hip, prescaled, fm)
            mks = [packed_full] if packed_full is not None else None  # backward packs its own (cached)
        # the score buffers travel as saved tensors: autograd frees them after the backward unless
        # the graph is retained (a ctx attribute would keep 20-40 GB alive as long as the graph is
        # referenced, e.g. through the previous step's loss)
        sbt = tuple(t for t in (sbuf, dsbuf) if t is not None)
        ctx.save_for_backward(k, o, lse, *bufs, *sbt)
        ctx.mks, ctx.mask, ctx.chunks, ctx.H, ctx.scale, ctx.comm, ctx.use_hip = mks, mask, chunks, H, scale, comm, use_hip
        ctx.prescaled, ctx.fp32_mode = prescaled, fm
        # (has S buffer, has dS buffer); the in-place mode (S only) is consumed by the first backward
        ctx.sb_kind = (sbuf is not None, dsbuf is not None)
        return o

    @staticmethod
    @_ext.pinned
    def backward(ctx, do):
        k, o, lse, *bufs = ctx.saved_tensors
        has_s, has_ds = getattr(ctx, "sb_kind", (False, False))
        nsb = int(has_s) + int(has_ds)
        sbt = bufs[len(bufs) - nsb:] if nsb else []
        bufs = bufs[:len(bufs) - nsb]
        comm, H, scale, chunks = ctx.comm, ctx.H, ctx.scale, ctx.chunks
        n = comm.world_size
        C = k.shape[-1]
        B, R = k.shape[0], k.shape[1]
        do = do.contiguous()

        def reduce_async(parts, out=None):  # (N, B, rc, 2C) rank-major partials -> (B, rc, 2C)
            if n == 1:
                return None, parts[0]
            if out is None:
                out = torch.empty(parts.shape[1:], dtype=parts.dtype, device=parts.device)
            return comm.reduce_scatter(out, parts, async_op=True), out

        if ctx.use_hip:
            from ..ops import flash

            one = len(bufs) == 1  # one gathered buffer: natural order, or chunks permuted (B = 1)
            mks = ctx.mks
            if mks is None or (one and len(chunks) > 1):  # segmented forward: masks packed here (cached)
                if one:
                    mks = [flash.prepare_mask_cached(ctx.mask, B, R, n * R,
                                                     tag=None if len(chunks) == 1 else ("perm", tuple(chunks), n),
                                                     view=None if len(chunks) == 1 else _perm_cols(B, R, n, chunks))]
                else:
                    mks = [flash.prepare_mask_cached(ctx.mask, B, R, n * rc, tag=(r0, rc, n),
                                                     view=_mask_cols(B, R, n, 0, n, r0, rc)) for r0, rc in chunks]
            # δ, then two independent streams: 1) gathered-side grads on a HIGH-priority stream,
            # followed there by their reduce-scatter(s), and 2) the row-side dk on the current
            # stream.  2) fills the partly occupied last workgroup rounds of 1) and hides the
            # reduce-scatter, while the priority keeps 1) (and so the collective) nearly as
            # early as when it runs alone.  δ runs on the priority stream too, so 1) reaches
            # the GPU first.  Per-chunk kernels (chunk c's reduce-scatter under chunk c+1's
            # kernel) only when the chunks are separate buffers (B > 1).
            cur = torch.cuda.current_stream(do.device)
            # high priority so the gathered side (and its reduce-scatter) finishes early (an
            # ordinary-priority side stream measured slower at N=1 and N=8: profiles/r2_bwd_overlap.md)
            hi = _side_stream(do.device, -1) if _two_stream_backward(R) else cur
            hi.wait_stream(cur)
            handles, outs = [], []
            gdt = k.dtype if not FLAGS.grad_fp32 else torch.float32
            # score buffer: S -> dS in the column kernel, then dK from dS.  With a separate dS buffer
            # S stays intact, so a second backward through a retained graph reads it again; in place
            # (S overwritten with dS) the first backward consumes it and a second one recomputes
            sbuf = sbt[0] if has_s else None
            dsbuf = sbt[-1] if has_ds else None
            if has_s and not has_ds:
                if getattr(ctx, "sb_used", False):
                    sbuf = None
                ctx.sb_used = True
            if (sbuf is None and k.dtype == torch.float32 and C // H > WIDE_F32_NEEDS_SCORES
                    and ctx.fp32_mode == 0):
                raise RuntimeError(
                    f"xdot: a second backward through a retained graph of exact-fp32 attention at head dim "
                    f"{C // H} needs the scores, which the first backward overwrote in place (no kernel "
                    "recomputes an fp32 head this wide); set XDOT_FP32_SCORES_DS=1 with room for the "
                    "separate dS buffer, or do not retain the graph")
            ev_cols = None
            with _on_stream(hi, cur):
                delta, lse2 = flash.bwd_prep(do, o, lse, H)  # one prep pass for both kernels
                ev = _prep_event(hi.device)
                ev.record(hi)
                dqv = None
                if n > 1 and len(chunks) > 1 and B == 1:
                    dqv = torch.empty(B, R, 2 * C, dtype=gdt, device=k.device)
                # partials rounded once to the compute dtype in the kernel (XDOT_GRAD_FP32=1
                # keeps fp32): half the epilogue stores and half the reduce-scatter bytes
                if one:
                    g = bufs[0]
                    cargs = dict(fp32_out=FLAGS.grad_fp32, prescaled=ctx.prescaled, lse2=lse2,
                                 fp32_mode=ctx.fp32_mode, sbuf=sbuf)
                    if dsbuf is not None and sbuf is not None:
                        # dQ pass (S -> dS), then the row kernel (reads dS) on `cur` concurrently
                        # with the dV pass (reads S) here.  (The dV pass beside the dQ pass on a third
                        # stream instead measured 54.62 vs 54.71 ms, and one rep ran 171 ms:
                        # profiles/r6_fp32.md)
                        dkv, _ = flash.bwd_cols(do, k, g[..., :C], g[..., C:], o, lse, mks[0], H, scale, delta,
                                                dsbuf=dsbuf, passes=2, **cargs)
                        ev_cols = torch.cuda.Event()
                        ev_cols.record(hi)
                        flash.bwd_cols(do, k, g[..., :C], g[..., C:], o, lse, mks[0], H, scale, delta,
                                       dsbuf=dsbuf, passes=1, out_dkv=dkv, **cargs)
                    else:
                        # (fused exact pass: dP, dQ and dV in one kernel, S -> dS in place)
                        fused = sbuf is not None and dsbuf is None and flash.fused_cols_wanted(ctx.fp32_mode, C // H)
                        dkv, _ = flash.bwd_cols(do, k, g[..., :C], g[..., C:], o, lse, mks[0], H, scale, delta,
                                                dsbuf=dsbuf, passes=4 if fused else 3, **cargs)
                        if sbuf is not None or dsbuf is not None:  # the row kernel reads the dS this kernel wrote
                            ev_cols = torch.cuda.Event()
                            ev_cols.record(hi)
                    off = 0
                    for r0, rc in chunks:  # (chunk, rank, row) order: chunk c's ranks are contiguous
                        part = dkv if len(chunks) == 1 else dkv[:, off:off + n * rc]
                        off += n * rc
                        h, oc = reduce_async(flash.btc_to_rank_major(part, n),
                                             None if dqv is None else dqv[:, r0:r0 + rc])
                        handles.append(h)
                        outs.append(oc)
                else:
                    for c, (r0, rc) in enumerate(chunks):
                        g = bufs[c]
                        dkv, _ = flash.bwd_cols(do, k, g[..., :C], g[..., C:], o, lse, mks[c], H, scale, delta,
                                                fp32_out=FLAGS.grad_fp32, prescaled=ctx.prescaled, lse2=lse2,
                                            fp32_mode=ctx.fp32_mode)
                        h, oc = reduce_async(flash.btc_to_rank_major(dkv, n),
                                             None if dqv is None else dqv[:, r0:r0 + rc])
                        handles.append(h)
                        outs.append(oc)
            # the row-side kernel starts as soon as δ exists: back to back measured slower at
            # every rank shape (profiles/r2_bwd_overlap.md)
            cur.wait_event(ev if ev_cols is None else ev_cols)
            delta.record_stream(cur)
            if one:
                g = bufs[0]
                dk = flash.bwd_rows(do, k, g[..., :C], g[..., C:], lse, delta, mks[0], H, scale,
                                    nsplit=FLAGS.rows_split, prescaled=ctx.prescaled, fp32_mode=ctx.fp32_mode,
                                    sbuf=sbuf, dsbuf=dsbuf)
                if sbuf is not None:
                    sbuf.record_stream(cur)
                if dsbuf is not None:
                    dsbuf.record_stream(cur)
            else:
                ops = _ext.ops()
                ns = int(ops.flash_splits(B, R, n * chunks[0][1], H, True))
                dpart = torch.empty(len(chunks) * ns, B, R, C, dtype=torch.float32, device=k.device)
                for c in range(len(chunks)):
                    g = bufs[c]
                    mk = mks[c]
                    bits, flags = (mk.bits, mk.flags) if mk is not None else (None, None)
                    ops.flash_bwd_rows_partial(do, k, flash._kv(g[..., :C]), flash._kv(g[..., C:]), lse, delta, bits,
                                               flags, int(H), float(scale), dpart, c * ns, ns, ctx.prescaled,
                                               ctx.fp32_mode)
                dk = ops.flash_bwd_rows_sum(dpart, int(H), k)
            with _on_stream(hi, cur):  # the gathered-side grads complete on the priority stream
                for h in handles:
                    if h is not None:
                        h.wait()
                handles = []
                if dqv is None:
                    dqv = outs[0] if len(outs) == 1 else torch.cat(outs, dim=1)
            cur.wait_stream(hi)
            for oc in outs:
                oc.record_stream(cur)
            dqv.record_stream(cur)
            # consumers that can run on the priority stream (the packed [q|v] projection's
            # weight gradient, xdot.ops.linear.LinearFn) start there as soon as the
            # reduce-scatter lands, under the row-side kernel still running on `cur`
            if FLAGS.wgrad_side and dqv.dtype == k.dtype:
                dqv._xdot_ready_on = hi
        else:
            qvg = bufs[0]
            dk, dq_parts, dv_parts = _ref_bwd(do, k, qvg[..., :C], qvg[..., C:], o, lse, ctx.mask, H, scale)
            parts = torch.cat([dq_parts, dv_parts], dim=-1)
            if k.dtype in (torch.bfloat16, torch.float16) and not FLAGS.grad_fp32:
                parts = parts.to(k.dtype)  # the HIP path's wire dtype (one rounding per partial)
            h, dqv = reduce_async(parts)
            handles = [h]
        for h in handles:
            if h is not None:
                h.wait()
        return dk.to(k.dtype), dqv.to(k.dtype), None, None, None, None, None, None, None


def gather_plan(qv_shape, qv: Tensor, comm: _comm.Communicator, chunks: Optional[int] = None):
    """Row chunks of the gathered side's pipeline for a (B, R, C) ``qv`` of this rank."""
    hip = _ext.use_hip(qv) and qv.dtype in FLASH_DTYPES
    return _row_chunks(comm.world_size, qv_shape[1], hip, chunks)


def start_gather(qv: Tensor, comm: Optional[_comm.Communicator] = None,
                 chunks: Optional[int] = None, out: Optional[Tensor] = None) -> "_PendingGather":
    """Issue the all-gather(s) of the packed gathered side early (e.g. before the row-side
    projection GEMM) and hand the result to :func:`seq_parallel_attention_packed`.
    ``chunks``: row chunks of the pipeline (default ``XDOT_GATHER_CHUNKS``).  ``out``: the
    (N, B, R, C) gather output whose block ``rank`` IS ``qv`` (the projection wrote it in place;
    one-chunk plans only)."""
    comm = comm or _comm.get_comm()
    plan = gather_plan(qv.shape, qv, comm, chunks)
    if out is not None and len(plan) != 1:
        raise ValueError("start_gather: an in-place output needs a one-chunk plan")
    return _PendingGather(comm, qv.detach(), plan, out=out)


def seq_parallel_attention_packed(k: Tensor, qv: Tensor, mask: Optional[Tensor], num_heads: int, scale: float,
                                  comm: Optional[_comm.Communicator] = None,
                                  pending: Optional["_PendingGather"] = None) -> Tensor:
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
        if isinstance(mask, torch.Tensor):
            mask = mask.to(torch.bool)
    return SeqParallelAttention.apply(k, qv, mask, num_heads, float(scale), comm, pending, False,
                                      torch.is_grad_enabled())


def seq_parallel_attention(k: Tensor, q: Tensor, v: Tensor, mask: Optional[Tensor], num_heads: int,
                           scale: float, comm: Optional[_comm.Communicator] = None) -> Tensor:
    """Fused sequence-parallel attention on projected, head-interleaved (B, R, H*d) tensors.

    ``k``: row side (local rows), ``q``/``v``: gathered side (local shards), ``mask``: bool
    (B, R, T) with True = masked, or None.  Returns (B, R, H*dv) in ``k``'s dtype.
    """
    if k.dim() != 3 or q.dim() != 3 or v.dim() != 3:
        raise ValueError("seq_parallel_attention expects (B, R, H*d) tensors")
    return seq_parallel_attention_packed(k, torch.cat([q, v], dim=-1), mask, num_heads, scale, comm)
