"""Ring ("offset-chunk exchange") sequence-parallel attention over point-to-point RCCL hops.

The reference moves the gathered side of every product in ``offset``-row chunks, each an
all-gather (``functions.py:69-97`` for ``nt``, ``:186-208`` for ``all``), and gathers again in
backward.  The default fused path (:mod:`xdot.parallel.attention`) replaces that
with ONE all-gather of the packed ``[q | v]`` — on MI355X's fully connected xGMI mesh an
all-gather drives all 7 links of a GPU at once, so it is the fastest way to move the whole
gathered side.

This module is the memory-lean alternative for sequences whose gathered side should never be
resident in full: the ``[q | v]`` shards travel around the ring one rank-block at a time
(``sendrecv`` to rank+1 / from rank-1 on the RCCL stream), and the block that arrived last step
is consumed by the flash kernels while the next one is in flight.  Resident per rank: two
``(B, R, 2C)`` blocks (instead of ``(B, T, 2C)``) plus ``1 + splits`` fp32 ``(B, R, C)`` partial
slots (a running merge: independent of the ring length).

forward   step s (s = 0..N-1) consumes block ``src = (rank - s) mod N``: the flash kernel
          writes its split partials (O, LSE), which are merged at once into a running fp32
          (O, LSE) slot; the last step's combine writes the output (blocks whose rows are fully
          masked contribute nothing, rows masked everywhere come out NaN like the reference);
backward  the blocks circulate again.  Per step: the row-side partial ``dk`` (summed once at
          the end) and the block's ``[dq | dv]`` contribution, added to an fp32 accumulator that
          travels WITH the block one hop behind it; after N steps plus one hop every rank holds
          the full gradient of its own block — no reduce-scatter.

Per hop one link carries ``R·2C`` bf16 (block) and ``R·2C`` fp32 (accumulator), so a ring is
link-bound where the all-gather is mesh-bound: it is selected explicitly
(``DistributedDotProductAttn(impl="ring")`` / :func:`ring_attention`), never by ``auto``.
CPU tensors (and dtypes the kernels do not take) run the same schedule with torch math.
"""
from __future__ import annotations

from typing import List, Optional

import torch
from torch import Tensor

from .. import _ext
from ..utils import comm as _comm
from ..utils.checks import check_consistent
from ..utils.env import FLAGS

__all__ = ["RingAttention", "ring_attention", "ring_attention_packed"]


def _heads(x: Tensor, H: int, cdt) -> Tensor:
    B, L, C = x.shape
    return x.view(B, L, H, C // H).transpose(1, 2).to(cdt)


def _ref_block_fwd(k, blk, mask, H, scale):
    """Block partial: (o (B, H, R, dv) normalised within the block, lse (B, H, R)), compute dtype."""
    cdt = torch.float64 if k.dtype == torch.float64 else torch.float32
    C = k.shape[-1]
    kh, qh, vh = _heads(k, H, cdt), _heads(blk[..., :C], H, cdt), _heads(blk[..., C:], H, cdt)
    s = torch.matmul(kh, qh.transpose(-1, -2)) * scale
    if mask is not None:
        s = s.masked_fill(mask.unsqueeze(1), -float("inf"))
    lse = torch.logsumexp(s, dim=-1)
    p = torch.exp(s - lse.unsqueeze(-1))
    return torch.matmul(p, vh), lse


def _ref_block_bwd(do, k, blk, lse, delta, mask, H, scale):
    """-> (dk (B, R, C), [dq | dv] of the block (B, R, 2C)), compute dtype."""
    cdt = lse.dtype
    B, R, C = k.shape
    kh, qh, vh = _heads(k, H, cdt), _heads(blk[..., :C], H, cdt), _heads(blk[..., C:], H, cdt)
    doh = _heads(do, H, cdt)
    s = torch.matmul(kh, qh.transpose(-1, -2)) * scale
    if mask is not None:
        s = s.masked_fill(mask.unsqueeze(1), -float("inf"))
    p = torch.exp(s - lse.unsqueeze(-1))
    ds = p * (torch.matmul(doh, vh.transpose(-1, -2)) - delta.unsqueeze(-1)) * scale
    merge = lambda x: x.transpose(1, 2).reshape(B, x.shape[2], -1)  # noqa: E731
    dk = merge(torch.matmul(ds, qh))
    dq = merge(torch.matmul(ds.transpose(-1, -2), kh))
    dv = merge(torch.matmul(p.transpose(-1, -2), doh))
    return dk, torch.cat([dq, dv], dim=-1)


class _Ring:
    """Double-buffered block ring: ``cur`` is consumed while ``nxt`` is being received.  The
    caller's ``first`` block is only ever sent, never received into (it is a saved tensor)."""

    def __init__(self, comm, first: Tensor):
        self.comm, self.n, self.rank = comm, comm.world_size, comm.rank
        self.first = first
        self.cur = first
        self.nxt = torch.empty_like(first) if self.n > 1 else None
        self.h = None

    def src(self, s: int) -> int:
        return (self.rank - s) % self.n

    def start(self, s: int):
        if s < self.n - 1:
            self.h = self.comm.sendrecv(self.cur, self.nxt, (self.rank + 1) % self.n, (self.rank - 1) % self.n,
                                        async_op=True)

    def advance(self):
        if self.h is not None:
            self.h.wait()
            self.h = None
            old, self.cur = self.cur, self.nxt
            self.nxt = torch.empty_like(old) if old is self.first else old


def _block_mask(mask: Optional[Tensor], src: int, R: int) -> Optional[Tensor]:
    return None if mask is None else mask[..., src * R:(src + 1) * R]


class RingAttention(torch.autograd.Function):
    """Ring attention on the packed gathered side ``qv = [q | v]`` (B, R, 2C) of this rank."""

    @staticmethod
    @_ext.pinned
    def forward(ctx, k, qv, mask, H, scale, comm):
        check_consistent(comm, "ring_attention", k, qv, H)
        B, R, C = k.shape
        n = comm.world_size
        from .attention import FLASH_DTYPES, FLASH_HEAD_DIMS

        use_hip = (_ext.use_hip(k) and k.dtype in FLASH_DTYPES and qv.shape[-1] == 2 * C
                   and C // H in FLASH_HEAD_DIMS)
        qv = qv.contiguous()
        ring = _Ring(comm, qv)
        mks: List = []
        prescaled = False
        fm = 0
        if use_hip:
            from ..ops import flash

            ops = _ext.ops()
            fm = flash.fp32_code(k.dtype)
            prescaled = FLAGS.prescale and (k.numel() % 8 == 0) and k.dtype != torch.float32
            kk = flash.prescale(k, scale) if prescaled else k.contiguous()
            ns = int(ops.flash_splits(B, R, R, H, False))
            # slot 0: the running (O, LSE) of the blocks seen so far (fp32), slots 1..ns: the
            # arriving block's split partials, merged into slot 0 after each step — resident
            # partials stay (1 + ns) slots whatever the ring length
            opart = torch.empty(1 + ns, B, R, C, dtype=torch.float32, device=k.device)
            lpart = torch.empty(1 + ns, B, H, R, dtype=torch.float32, device=k.device)
            lpart[0].fill_(-float("inf"))
            lrun = torch.empty(B, H, R, dtype=torch.float32, device=k.device)
            for s in range(n):
                ring.start(s)
                src = ring.src(s)
                mk = flash.prepare_mask_cached(mask, B, R, R, tag=("ring", src, R),
                                               view=lambda m, src=src: _block_mask(m, src, R))
                mks.append(mk)
                bits, flags = (mk.bits, mk.flags) if mk is not None else (None, None)
                g = ring.cur
                ops.flash_fwd_partial(kk, flash._kv(g[..., :C]), flash._kv(g[..., C:]), bits, flags, int(H),
                                      float(scale), opart, lpart, 1, ns, prescaled, fm)
                if s < n - 1:
                    ops.flash_fwd_merge(opart, lpart, lrun, int(H))
                    lpart[0].copy_(lrun)
                ring.advance()
            o, lse = ops.flash_fwd_combine(opart, lpart, int(H), k)
            ctx.save_for_backward(kk, qv, o, lse)
        else:
            cdt = torch.float64 if k.dtype == torch.float64 else torch.float32
            acc = torch.zeros(B, H, R, (qv.shape[-1] - C) // H, dtype=cdt, device=k.device)
            lse = torch.full((B, H, R), -float("inf"), dtype=cdt, device=k.device)
            for s in range(n):
                ring.start(s)
                m = _block_mask(mask, ring.src(s), R)
                mks.append(m)
                ob, lb = _ref_block_fwd(k, ring.cur, m, H, scale)
                new = torch.logaddexp(lse, lb)
                live = torch.isfinite(new).unsqueeze(-1)
                w_old = torch.where(live, torch.exp(lse - new).unsqueeze(-1), torch.zeros_like(acc[..., :1]))
                w_new = torch.where(torch.isfinite(lb).unsqueeze(-1), torch.exp(lb - new).unsqueeze(-1),
                                    torch.zeros_like(acc[..., :1]))
                acc = acc * w_old + torch.nan_to_num(ob, nan=0.0) * w_new
                lse = new
                ring.advance()
            acc = torch.where(torch.isfinite(lse).unsqueeze(-1), acc, torch.full_like(acc, float("nan")))
            o = acc.transpose(1, 2).reshape(B, R, -1).to(k.dtype)
            ctx.save_for_backward(k, qv, o, lse)
        ctx.mks, ctx.H, ctx.scale, ctx.comm, ctx.use_hip, ctx.prescaled = mks, H, scale, comm, use_hip, prescaled
        ctx.fp32_mode = fm
        return o

    @staticmethod
    @_ext.pinned
    def backward(ctx, do):
        k, qv, o, lse = ctx.saved_tensors
        comm, H, scale = ctx.comm, ctx.H, ctx.scale
        n, rank = comm.world_size, comm.rank
        B, R, C = k.shape
        do = do.contiguous()
        ring = _Ring(comm, qv)
        acc_in = torch.empty(B, R, qv.shape[-1], dtype=torch.float32 if k.dtype != torch.float64 else k.dtype,
                             device=k.device) if n > 1 else None
        acc_h = None
        acc = None
        if ctx.use_hip:
            from ..ops import flash

            from .attention import _side_stream

            ops = _ext.ops()
            cur = torch.cuda.current_stream(do.device)
            ov = FLAGS.ring_overlap
            two = ov not in ("0", "false", "off", "no") and (ov != "auto" or -(-R // 128) * B * H >= 1024)
            hi = _side_stream(do.device) if two else cur  # XDOT_RING_OVERLAP (utils/env.py)
            delta = flash.bwd_delta(do, o, H)
            nsr = int(ops.flash_splits(B, R, R, H, True))
            # slot 0: running fp32 dk, slots 1..nsr: this step's column-split partials
            dpart = torch.empty(1 + nsr, B, R, C, dtype=torch.float32, device=k.device)
            dpart[0].zero_()
        else:
            cdt = lse.dtype
            delta = (_heads(do, H, cdt) * _heads(o, H, cdt)).sum(-1)
            dk = torch.zeros(B, R, C, dtype=cdt, device=k.device)
        for s in range(n):
            ring.start(s)
            g = ring.cur
            mk = ctx.mks[s]
            if ctx.use_hip:
                # the gathered-side kernel runs on the high-priority side stream, concurrently
                # with the row-side partial here, when a block is big enough for that to pay
                # (``hi is cur`` otherwise)
                hi.wait_stream(cur)
                with torch.cuda.stream(hi):
                    contrib, _ = flash.bwd_cols(do, k, g[..., :C], g[..., C:], o, lse, mk, H, scale, delta,
                                                fp32_out=True, prescaled=ctx.prescaled, fp32_mode=ctx.fp32_mode)
                bits, flags = (mk.bits, mk.flags) if mk is not None else (None, None)
                ops.flash_bwd_rows_partial(do, k, flash._kv(g[..., :C]), flash._kv(g[..., C:]), lse, delta, bits,
                                           flags, int(H), float(scale), dpart, 1, nsr, ctx.prescaled,
                                           ctx.fp32_mode)
                if s < n - 1:
                    ops.sum_partials_into(dpart, dpart[0])
                cur.wait_stream(hi)
                contrib.record_stream(cur)
            else:
                dkb, contrib = _ref_block_bwd(do, k, g, lse, delta, mk, H, scale)
                dk += dkb
                contrib = contrib.to(acc_in.dtype if acc_in is not None else contrib.dtype)
            # the accumulator of this block arrives from rank-1 one hop behind the block itself
            if acc_h is not None:
                acc_h.wait()
                contrib += acc_in
            acc = contrib
            if n > 1:  # acc_in was consumed above (stream-ordered before the receive overwrites it)
                acc_h = comm.sendrecv(acc, acc_in, (rank + 1) % n, (rank - 1) % n, async_op=True)
            ring.advance()
        if acc_h is not None:
            acc_h.wait()
            acc = acc_in
        if ctx.use_hip:
            dk = ops.flash_bwd_rows_sum(dpart, int(H), k)
        return dk.to(k.dtype), acc.to(k.dtype), None, None, None, None


def ring_attention_packed(k: Tensor, qv: Tensor, mask: Optional[Tensor], num_heads: int, scale: float,
                          comm: Optional[_comm.Communicator] = None) -> Tensor:
    """Ring sequence-parallel attention with a packed gathered side ``qv = [q | v]`` (B, R, C + Cv);
    ``mask``: bool (B, R, T) (True = masked) or None.  Returns (B, R, Cv) in ``k``'s dtype."""
    comm = comm or _comm.get_comm()
    if k.dim() != 3 or qv.dim() != 3 or qv.shape[-1] <= k.shape[-1] or qv.shape[:2] != k.shape[:2]:
        raise ValueError("ring_attention expects k (B, R, C) and qv (B, R, C + Cv) with equal R")
    if mask is not None:
        T = qv.shape[1] * comm.world_size
        if tuple(mask.shape) != (k.shape[0], k.shape[1], T):
            raise ValueError(f"mask must be (B, R, T)=({k.shape[0]}, {k.shape[1]}, {T}), got {tuple(mask.shape)}")
        mask = mask.to(torch.bool)
    return RingAttention.apply(k, qv, mask, num_heads, float(scale), comm)


def ring_attention(k: Tensor, q: Tensor, v: Tensor, mask: Optional[Tensor], num_heads: int, scale: float,
                   comm: Optional[_comm.Communicator] = None) -> Tensor:
    """:func:`ring_attention_packed` on separate head-interleaved (B, R, H*d) ``k``, ``q``, ``v``."""
    return ring_attention_packed(k, torch.cat([q, v], dim=-1), mask, num_heads, scale, comm)
