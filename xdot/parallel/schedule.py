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
