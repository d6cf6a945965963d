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

Bidirectional (``XDOT_RING_BIDIR``, default on, N >= 3): rows ``[0, R/2)`` of every block travel
one way round the ring and rows ``[R/2, R)`` the other, so each hop drives two xGMI links (to
rank+1 and rank-1) with half the bytes each, and the backward accumulators travel in the compute
dtype (bf16: the same per-hop rounding as the fused path's reduce-scatter).  Per hop each of the
two links carries ``R/2·2C`` 16-bit elements (block) and as many again (accumulator).  A ring is
still link-bound where the all-gather is mesh-bound: it is selected explicitly
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
    """Double-buffered block ring of one direction (``d`` = +1: to rank+1 / from rank-1, -1: the
    other way): ``cur`` is consumed while ``nxt`` is being received.  The caller's ``first``
    block is only ever sent, never received into (it is a saved tensor)."""

    def __init__(self, comm, first: Tensor, d: int = 1):
        self.comm, self.n, self.rank, self.d = comm, comm.world_size, comm.rank, d
        self.first = first
        self.cur = first
        self.nxt = torch.empty_like(first) if self.n > 1 else None

    def src(self, s: int) -> int:
        """the rank whose block this ring holds at step s"""
        return (self.rank - self.d * s) % self.n

    def pair(self):
        return (self.cur, self.nxt, (self.rank + self.d) % self.n, (self.rank - self.d) % self.n)

    def rotate(self):
        old, self.cur = self.cur, self.nxt
        self.nxt = torch.empty_like(old) if old is self.first else old


class _Rings:
    """The lanes of one ring schedule, hopped together (one grouped exchange per step).

    With ``N >= 3`` ranks the block is split by rows: rows ``[0, R/2)`` travel one way round the
    ring and rows ``[R/2, R)`` the other, so every hop drives TWO xGMI links (to rank+1 and to
    rank-1) with half the bytes each: the hop takes half the time of a one-way ring.  Lane i is
    ``(d, a, b)``: direction and the block rows it carries.

    ``merged`` (B = 1): the two lanes' halves live in ONE (1, R, 2C) buffer per ring slot
    (``full_cur`` / ``full_nxt``), so each step's kernels run once over the whole block (columns
    [0, R/2) from one source rank, [R/2, R) from the other) -- as many launches per hop as the
    one-way ring, at full width."""

    def __init__(self, comm, blk: Tensor, bidir: bool):
        R = blk.shape[1]
        n = comm.world_size
        self.comm = comm
        if bidir and n >= 3 and R >= 2:
            h = R // 2
            self.lanes = [(1, 0, h), (-1, h, R)]
        else:
            self.lanes = [(1, 0, R)]
        self.merged = len(self.lanes) > 1 and blk.shape[0] == 1 and blk.is_contiguous()
        if self.merged:
            self.full_first = self.full_cur = blk
            self.full_nxt = torch.empty_like(blk)
            self.rings = [_Ring(comm, blk[:, a:b], d) for (d, a, b) in self.lanes]
            self._views()
        else:
            self.rings = [_Ring(comm, blk[:, a:b].contiguous() if len(self.lanes) > 1 else blk, d)
                          for (d, a, b) in self.lanes]
        self.h = None

    def _views(self):
        for r, (_d, a, b) in zip(self.rings, self.lanes):
            r.cur, r.nxt = self.full_cur[:, a:b], self.full_nxt[:, a:b]

    def start(self, s: int):
        if s < self.comm.world_size - 1:
            self.h = self.comm.sendrecv_multi([r.pair() for r in self.rings], async_op=True)

    def advance(self):
        if self.h is not None:
            self.h.wait()
            self.h = None
            if self.merged:
                old, self.full_cur = self.full_cur, self.full_nxt
                self.full_nxt = torch.empty_like(old) if old is self.full_first else old
                self._views()
            else:
                for r in self.rings:
                    r.rotate()

    def units(self, s: int, mask: Optional[Tensor], R: int):
        """The kernel launches of step s: ``[(block, mask view fn or None, tag, lanes)]`` -- one
        per lane, or one over the merged block (``lanes`` = the lane indices it covers)."""
        if self.merged:
            (_d0, _a0, h), _ = self.lanes
            s0, s1 = self.rings[0].src(s), self.rings[1].src(s)
            view = (lambda m, s0=s0, s1=s1: torch.cat([_block_mask(m, s0, R, 0, h), _block_mask(m, s1, R, h, R)], -1)) \
                if mask is not None else None
            return [(self.full_cur, view, ("ringm", s0, s1, h, R), (0, 1))]
        out = []
        for li, ((_d, a, b), ring) in enumerate(zip(self.lanes, self.rings)):
            src = ring.src(s)
            view = (lambda m, src=src, a=a, b=b: _block_mask(m, src, R, a, b)) if mask is not None else None
            out.append((ring.cur, view, ("ring", src, a, b, R), (li,)))
        return out


def _block_mask(mask: Optional[Tensor], src: int, R: int, a: int = 0, b: Optional[int] = None) -> Optional[Tensor]:
    b = R if b is None else b
    return None if mask is None else mask[..., src * R + a:src * R + b]


def _bidir() -> bool:
    return FLAGS.ring_bidir


class RingAttention(torch.autograd.Function):
    """Ring attention on the packed gathered side ``qv = [q | v]`` (B, R, 2C) of this rank."""

    @staticmethod
    @_ext.pinned
    def forward(ctx, k, qv, mask, H, scale, comm):
        check_consistent(comm, "ring_attention", k, qv, H)
        B, R, C = k.shape
        n = comm.world_size
        from .attention import FLASH_DTYPES, FLASH_HEAD_DIMS, WIDE_F32_NEEDS_SCORES

        # (the ring has no score buffer: exact fp32 heads past 256 run the torch path)
        use_hip = (_ext.use_hip(k) and k.dtype in FLASH_DTYPES and qv.shape[-1] == 2 * C
                   and C // H in FLASH_HEAD_DIMS
                   and not (k.dtype == torch.float32 and C // H > WIDE_F32_NEEDS_SCORES))
        qv = qv.contiguous()
        rings = _Rings(comm, qv, _bidir())
        L = len(rings.lanes)
        mks: List = []  # per step, per lane
        prescaled = False
        fm = 0
        if use_hip:
            from ..ops import flash

            ops = _ext.ops()
            fm = flash.fp32_code(k.dtype)
            prescaled = FLAGS.prescale and (k.numel() % 8 == 0) and k.dtype != torch.float32
            kk = flash.prescale(k, scale) if prescaled else k.contiguous()
            U = 1 if rings.merged else L  # kernel launches per step
            ns = int(ops.flash_splits(B, R, R if rings.merged else max(b - a for _, a, b in rings.lanes), H, False))
            # slot 0: the running (O, LSE) of the blocks seen so far (fp32), then ns slots per launch
            # for the arriving pieces' split partials, merged into slot 0 after each step -- resident
            # partials stay (1 + U ns) slots whatever the ring length
            opart = torch.empty(1 + U * ns, B, R, C, dtype=torch.float32, device=k.device)
            lpart = torch.empty(1 + U * ns, B, H, R, dtype=torch.float32, device=k.device)
            lpart[0].fill_(-float("inf"))
            lrun = torch.empty(B, H, R, dtype=torch.float32, device=k.device)
            for s in range(n):
                rings.start(s)
                step = []
                for ui, (g, view, tag, _lanes) in enumerate(rings.units(s, mask, R)):
                    mk = flash.prepare_mask_cached(mask, B, R, g.shape[1], tag=tag, view=view)
                    step.append(mk)
                    bits, flags = (mk.bits, mk.flags) if mk is not None else (None, None)
                    ops.flash_fwd_partial(kk, flash._kv(g[..., :C]), flash._kv(g[..., C:]), bits, flags, int(H),
                                          float(scale), opart, lpart, 1 + ui * ns, ns, prescaled, fm)
                mks.append(step)
                if s < n - 1:
                    ops.flash_fwd_merge(opart, lpart, lrun, int(H))
                    lpart[0].copy_(lrun)
                rings.advance()
            o, lse = ops.flash_fwd_combine(opart, lpart, int(H), k)
            ctx.save_for_backward(kk, qv, o, lse)
        else:
            cdt = torch.float64 if k.dtype == torch.float64 else torch.float32
            acc = torch.zeros(B, H, R, (qv.shape[-1] - C) // H, dtype=cdt, device=k.device)
            lse = torch.full((B, H, R), -float("inf"), dtype=cdt, device=k.device)
            for s in range(n):
                rings.start(s)
                step = []
                for (_d, a, b), ring in zip(rings.lanes, rings.rings):
                    m = _block_mask(mask, ring.src(s), R, a, b)
                    step.append(m)
                    ob, lb = _ref_block_fwd(k, ring.cur, m, H, scale)
                    new = torch.logaddexp(lse, lb)
                    live = torch.isfinite(new).unsqueeze(-1)
                    w_old = torch.where(live, torch.exp(lse - new).unsqueeze(-1), torch.zeros_like(acc[..., :1]))
                    w_new = torch.where(torch.isfinite(lb).unsqueeze(-1), torch.exp(lb - new).unsqueeze(-1),
                                        torch.zeros_like(acc[..., :1]))
                    acc = acc * w_old + torch.nan_to_num(ob, nan=0.0) * w_new
                    lse = new
                mks.append(step)
                rings.advance()
            acc = torch.where(torch.isfinite(lse).unsqueeze(-1), acc, torch.full_like(acc, float("nan")))
            o = acc.transpose(1, 2).reshape(B, R, -1).to(k.dtype)
            ctx.save_for_backward(k, qv, o, lse)
        ctx.mks, ctx.H, ctx.scale, ctx.comm, ctx.use_hip, ctx.prescaled = mks, H, scale, comm, use_hip, prescaled
        ctx.fp32_mode, ctx.bidir = fm, L > 1
        return o

    @staticmethod
    @_ext.pinned
    def backward(ctx, do):
        k, qv, o, lse = ctx.saved_tensors
        comm, H, scale = ctx.comm, ctx.H, ctx.scale
        n = comm.world_size
        B, R, C = k.shape
        do = do.contiguous()
        rings = _Rings(comm, qv, ctx.bidir)
        lanes = rings.lanes
        # the [dq | dv] accumulators travel one hop behind their blocks, in the compute dtype (as
        # the fused path's reduce-scatter; XDOT_GRAD_FP32=1 keeps fp32 on the wire) -- each rank
        # adds its fp32 contribution to the arriving partial sum before forwarding it
        wdt = k.dtype if (k.dtype in (torch.bfloat16, torch.float16) and not FLAGS.grad_fp32) else (
            torch.float32 if k.dtype != torch.float64 else k.dtype)
        acc_in = [torch.empty(B, b - a, qv.shape[-1], dtype=wdt, device=k.device) for (_d, a, b) in lanes] \
            if n > 1 else None
        acc_h = None
        accs = None
        if ctx.use_hip:
            from ..ops import flash

            from .attention import _side_stream

            ops = _ext.ops()
            cur = torch.cuda.current_stream(do.device)
            ov = FLAGS.ring_overlap
            two = ov not in ("0", "false", "off", "no") and (ov != "auto" or -(-R // 128) * B * H >= 1024)
            hi = _side_stream(do.device) if two else cur  # XDOT_RING_OVERLAP (utils/env.py)
            delta = flash.bwd_delta(do, o, H)
            U = 1 if rings.merged else len(lanes)  # kernel launches per step
            nsr = int(ops.flash_splits(B, R, R if rings.merged else max(b - a for _, a, b in lanes), H, True))
            # slot 0: running fp32 dk, then nsr column-split partial slots per launch
            dpart = torch.empty(1 + U * nsr, B, R, C, dtype=torch.float32, device=k.device)
            dpart[0].zero_()
        else:
            cdt = lse.dtype
            delta = (_heads(do, H, cdt) * _heads(o, H, cdt)).sum(-1)
            dk = torch.zeros(B, R, C, dtype=cdt, device=k.device)
        for s in range(n):
            rings.start(s)
            contribs = []
            if ctx.use_hip:
                # the gathered-side kernels run on the high-priority side stream, concurrently with
                # the row-side partials here, when a block is big enough for that to pay
                # (``hi is cur`` otherwise)
                units = rings.units(s, None, R)
                full = []
                hi.wait_stream(cur)
                with torch.cuda.stream(hi):
                    for ui, (g, _v, _t, ls) in enumerate(units):
                        c_, _ = flash.bwd_cols(do, k, g[..., :C], g[..., C:], o, lse, ctx.mks[s][ui], H, scale, delta,
                                               fp32_out=True, prescaled=ctx.prescaled, fp32_mode=ctx.fp32_mode)
                        full.append(c_)
                        # a merged launch covers both lanes: lane li's contribution is its row range
                        contribs.extend(c_ if len(ls) == 1 else c_[:, lanes[li][1]:lanes[li][2]] for li in ls)
                for ui, (g, _v, _t, _ls) in enumerate(units):
                    mk = ctx.mks[s][ui]
                    bits, flags = (mk.bits, mk.flags) if mk is not None else (None, None)
                    ops.flash_bwd_rows_partial(do, k, flash._kv(g[..., :C]), flash._kv(g[..., C:]), lse, delta, bits,
                                               flags, int(H), float(scale), dpart, 1 + ui * nsr, nsr, ctx.prescaled,
                                               ctx.fp32_mode)
                if s < n - 1:
                    ops.sum_partials_into(dpart, dpart[0])
                cur.wait_stream(hi)
                for c_ in full:
                    c_.record_stream(cur)
            else:
                for li, ring in enumerate(rings.rings):
                    dkb, c_ = _ref_block_bwd(do, k, ring.cur, lse, delta, ctx.mks[s][li], H, scale)
                    dk += dkb
                    contribs.append(c_)
            # each accumulator arrives from the previous rank of its lane one hop behind its block
            if acc_h is not None:
                acc_h.wait()
                for c_, ai in zip(contribs, acc_in):
                    c_ += ai
            accs = [c_.to(wdt) for c_ in contribs]
            if n > 1:  # acc_in was consumed above (stream-ordered before the receive overwrites it)
                acc_h = comm.sendrecv_multi([(a_, ai, (comm.rank + d) % n, (comm.rank - d) % n)
                                             for a_, ai, (d, _a, _b) in zip(accs, acc_in, lanes)], async_op=True)
            rings.advance()
        if acc_h is not None:
            acc_h.wait()
            accs = acc_in
        dqv = accs[0] if len(accs) == 1 else torch.cat(accs, dim=1)
        if ctx.use_hip:
            dk = ops.flash_bwd_rows_sum(dpart, int(H), k)
        return dk.to(k.dtype), dqv.to(k.dtype), None, None, None, None


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
