"""Chunk planning and the double-buffered gather pipeline shared by the distributed ops.

The reference loops over ``offset``-sized chunks, each a *blocking* Horovod all-gather
followed by a GEMM (reference: ``functions.py:89-97`` rows of ``right`` for ``nt``,
``:202-210`` feature columns for ``all``); communication and compute never overlap and each
chunk pays negotiation latency (≈20-50 ms per extra chunk on its hardware).

Here:

* ``offset=None`` (default) = one chunk per op: a single RCCL all-gather of the whole peer
  shard (e.g. 3125 rows x 768 bf16 = 4.8 MB per rank at T=25000/N=8), big enough to run
  the xGMI links at bandwidth rather than latency.  An explicit ``offset`` is honoured
  exactly (API parity, short last chunk allowed);
* with several chunks the gather of chunk i+1 is issued (async, on RCCL's stream) before the
  GEMM of chunk i and waited for on the compute stream only when needed — a two-deep
  ring of preallocated buffers, no host synchronisation;
* :func:`gather_rows_grouped` — the row-chunk plan of ``nt`` / ``all`` with small offsets: the
  per-chunk cost of the loop above is host work (a collective call and a GEMM launch per
  chunk: 98 chunks of 32 rows at T=25000, N=8), so consecutive chunks form groups: each chunk
  is still ONE all-gather of exactly its rows (the reference's granularity on the wire), but
  a group's gathers are issued together (one coalesced RCCL launch), land in one buffer and
  feed ONE GEMM, while the next group's gathers are in flight (two groups double-buffered,
  within ``XDOT_CHUNK_BUDGET_MB`` / a 256 MB default per group);
* :func:`auto_offset` sizes chunks from free HBM when the caller asks for ``offset='auto'``.
"""
from __future__ import annotations

from typing import Callable, List, Optional, Sequence, Tuple, Union

import torch

from ..utils.env import FLAGS

Offset = Optional[Union[int, str]]


def plan_chunks(total: int, offset: Optional[int]) -> List[Tuple[int, int]]:
    """Contiguous ``[start, stop)`` chunks of ``offset`` items (last one may be short)."""
    if total <= 0:
        return []
    if offset is None or offset >= total:
        return [(0, total)]
    if offset <= 0:
        raise ValueError(f"offset must be positive, got {offset}")
    return [(s, min(s + offset, total)) for s in range(0, total, offset)]


def free_hbm_bytes(device: torch.device) -> int:
    if device.type != "cuda":
        return 1 << 40
    free, _total = torch.cuda.mem_get_info(device)
    return int(free)


def auto_offset(total: int, bytes_per_item: int, device: torch.device, fraction: float = 0.25) -> int:
    """Largest chunk whose double-buffered gather fits ``fraction`` of free HBM
    (or ``XDOT_CHUNK_BUDGET_MB`` when set)."""
    budget = FLAGS.chunk_budget_mb * 2**20 if FLAGS.chunk_budget_mb > 0 else free_hbm_bytes(device) * fraction
    per = max(1, 2 * bytes_per_item)
    return max(1, min(total, int(budget // per)))


def resolve_offset(offset: Offset, total: int, bytes_per_item: int, device: torch.device) -> Optional[int]:
    if offset == "auto":
        o = auto_offset(total, bytes_per_item, device)
        return None if o >= total else o
    if offset is not None and not isinstance(offset, int):
        raise TypeError(f"offset must be int, None or 'auto', got {offset!r}")
    return offset


def gather_pipeline(comm, chunks: Sequence[Tuple[int, int]], make_send: Callable[[int, int], torch.Tensor],
                    buf_shape: Callable[[int], Tuple[int, ...]], dtype: torch.dtype, device: torch.device,
                    consume: Callable[[int, int, torch.Tensor], None]) -> None:
    """For every chunk: all-gather ``make_send(s, e)`` into a rank-major buffer and call
    ``consume(s, e, gathered)``.  Gather i+1 overlaps consume i (two rotating buffers)."""
    if not chunks:
        return
    n = comm.world_size
    maxlen = max(e - s for s, e in chunks)
    bufs = [torch.empty((n,) + tuple(buf_shape(maxlen)), dtype=dtype, device=device)
            for _ in range(min(2, len(chunks)))]

    def issue(i):
        s, e = chunks[i]
        send = make_send(s, e).contiguous()
        out = bufs[i % len(bufs)].view(-1)[: n * send.numel()].view((n,) + tuple(send.shape))
        return comm.all_gather_into(out, send, async_op=True), out

    pending = issue(0)
    for i, (s, e) in enumerate(chunks):
        nxt = issue(i + 1) if i + 1 < len(chunks) else None
        h, out = pending
        h.wait()
        consume(s, e, out)
        pending = nxt


GROUP_BYTES = 256 * 2**20


def gather_rows_grouped(comm, r3: torch.Tensor, chunks: Sequence[Tuple[int, int]],
                        consume: Callable[[int, int, torch.Tensor], None]) -> None:
    """Row chunks ``[s, e)`` of ``r3`` (Pn, Rr, D), each gathered by its own all-gather, consumed
    in groups: ``consume(s0, e0, gathered)`` with ``gathered`` (N, Pn, e0 - s0, D) rank-major,
    the rows of a whole group of consecutive chunks (at least two groups when there are at
    least two chunks, so a group's GEMM overlaps the next group's gathers)."""
    if not chunks:
        return
    n = comm.world_size
    Pn, Rr, D = r3.shape
    if n == 1:  # nothing travels: one consumer call over every row
        consume(0, Rr, r3.unsqueeze(0))
        return
    rt = (r3[0] if Pn == 1 else r3.transpose(0, 1)).contiguous()  # (Rr, [Pn,] D): chunk rows contiguous
    row_bytes = n * Pn * D * r3.element_size()
    budget = FLAGS.chunk_budget_mb * 2**20 / 4 if FLAGS.chunk_budget_mb > 0 else GROUP_BYTES
    c = max(e - s for s, e in chunks)
    per_group = max(1, min(-(-len(chunks) // 2), int(budget // max(1, c * row_bytes))))
    groups = [list(chunks[i:i + per_group]) for i in range(0, len(chunks), per_group)]
    maxrows = max(g[-1][1] - g[0][0] for g in groups)
    nslot = min(2, len(groups))
    raws = [torch.empty(n * maxrows * Pn * D, dtype=r3.dtype, device=r3.device) for _ in range(nslot)]
    dests = [torch.empty(n * Pn * maxrows * D, dtype=r3.dtype, device=r3.device) for _ in range(nslot)]

    def issue(g):
        grp = groups[g]
        s0, e0 = grp[0][0], grp[-1][1]
        raw = raws[g % nslot][:n * (e0 - s0) * Pn * D]
        return comm.all_gather_chunks(raw, rt[s0:e0], [e - s for s, e in grp], async_op=True), raw

    pend = issue(0)
    for g, grp in enumerate(groups):
        nxt = issue(g + 1) if g + 1 < len(groups) else None
        h, raw = pend
        h.wait()
        s0, e0 = grp[0][0], grp[-1][1]
        dest = dests[g % nslot][:n * Pn * (e0 - s0) * D].view(n, Pn, e0 - s0, D)
        off = r = 0
        for cc, cnt in _runs([e - s for s, e in grp]):  # (cnt, N, cc, Pn, D) -> (N, Pn, cnt*cc, D)
            seg = raw[off:off + cnt * n * cc * Pn * D].view(cnt, n, cc, Pn, D)
            dest[:, :, r:r + cnt * cc].unflatten(2, (cnt, cc)).copy_(seg.permute(1, 3, 0, 2, 4))
            off += cnt * n * cc * Pn * D
            r += cnt * cc
        consume(s0, e0, dest)
        pend = nxt


def gather_rows_whole(comm, r3: torch.Tensor, chunks: Sequence[Tuple[int, int]]) -> torch.Tensor:
    """Every row chunk of ``r3`` (Pn, Rr, D) all-gathered by its own collective (grouped launches,
    all in flight together) into ONE (Pn, N*Rr, D) buffer in global row order: the B operand of
    ``all``'s single K = T GEMM.  Each group is reordered as soon as it lands, under the
    transfers of the later groups."""
    n = comm.world_size
    Pn, Rr, D = r3.shape
    if n == 1:
        return r3
    if len(chunks) == 1 and (Pn == 1 or r3.transpose(0, 1).is_contiguous()):
        # one gather of the (Rr, Pn*D) rows as they are: (N*Rr, Pn, D) is already global row
        # order, handed out as a (Pn, T, D) view (row stride Pn*D) for the GEMM to read in place
        dest = torch.empty(n * Rr * Pn * D, dtype=r3.dtype, device=r3.device)
        comm.all_gather_into(dest.view(n, Rr, Pn, D), r3.transpose(0, 1).contiguous())
        return dest.view(n * Rr, Pn, D).transpose(0, 1)
    rt = (r3[0] if Pn == 1 else r3.transpose(0, 1)).contiguous()
    row_bytes = n * Pn * D * r3.element_size()
    budget = FLAGS.chunk_budget_mb * 2**20 / 4 if FLAGS.chunk_budget_mb > 0 else GROUP_BYTES
    c = max(e - s for s, e in chunks)
    per_group = max(1, min(-(-len(chunks) // 2), int(budget // max(1, c * row_bytes))))
    groups = [list(chunks[i:i + per_group]) for i in range(0, len(chunks), per_group)]
    raw_all = torch.empty(n * Rr * Pn * D, dtype=r3.dtype, device=r3.device)
    pend, off = [], 0
    for grp in groups:
        s0, e0 = grp[0][0], grp[-1][1]
        raw = raw_all[off:off + n * (e0 - s0) * Pn * D]
        off += raw.numel()
        pend.append((comm.all_gather_chunks(raw, rt[s0:e0], [e - s for s, e in grp], async_op=True), raw))
    dest = torch.empty(Pn, n, Rr, D, dtype=r3.dtype, device=r3.device)
    for grp, (h, raw) in zip(groups, pend):
        h.wait()
        o = 0
        r = grp[0][0]
        for cc, cnt in _runs([e - s for s, e in grp]):  # (cnt, N, cc, Pn, D) -> (Pn, N, cnt*cc, D)
            seg = raw[o:o + cnt * n * cc * Pn * D].view(cnt, n, cc, Pn, D)
            dest[:, :, r:r + cnt * cc].unflatten(2, (cnt, cc)).copy_(seg.permute(3, 1, 0, 2, 4))
            o += cnt * n * cc * Pn * D
            r += cnt * cc
    return dest.view(Pn, n * Rr, D)


def _runs(sizes):
    out = []
    for c in sizes:
        if out and out[-1][0] == c:
            out[-1][1] += 1
        else:
            out.append([c, 1])
    return out
