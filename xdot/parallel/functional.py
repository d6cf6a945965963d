"""Sequence-parallel distributed products (time axis sharded into contiguous T/N row blocks).

Rank ``r`` holds global rows ``[r*R, (r+1)*R)`` (``R = T/N``, equal on all ranks) of every
sequence tensor; arbitrary identical leading dims ``P`` are allowed.  Contract (SURVEY §2.5,
reference ``distributed_dot_product/multiplication/functions.py``):

==============================  ==============  ==========  ===================================
function                        local inputs    local out   global math (row block ``r``)
==============================  ==============  ==========  ===================================
``distributed_matmul_nt``       (P,R,D),(P,R,D)  (P,R,T)     L·Rᵀ, column ``j*R+i`` = rank j row i
``distributed_matmul_all``      (P,R,T),(P,R,D)  (P,R,D)     L·R
``distributed_matmul_tn``       (P,R,T),(P,R,D)  (P,R,D)     Lᵀ·R
``distributed_matmul_block``    (P,R,K),(P,K,M)  (P,R,M)     Σ_ranks L_r·R_r  (Sum all-reduce)
==============================  ==============  ==========  ===================================

MI355X design, per op:

* ``nt`` (reference :45-99): RCCL all-gather of ``right`` (whole shard by default, or
  ``offset``-row chunks, double-buffered), then ONE batched MFMA GEMM per chunk over
  (source rank, P) that writes straight into the final (P, R, T) layout — no ``(N,P,R,R)``
  staging buffer and no permute copy (reference K3/K4).  Optional ``alpha`` fuses the
  attention scale into the epilogue.
* ``all`` (reference :161-212): all-gather ``right``, then one GEMM whose K loop walks the N
  source-rank column blocks of ``left`` in place — the reference's full ``torch.stack`` copy
  of ``left`` (7.5 GB at T=75000) and the trailing ``sum(dim=0)`` are gone.  With an
  ``offset`` the gather buffer keeps the reference's size (N·R·offset elements) but holds
  whole rows of ``right``, accumulated over K steps, so ``left`` is read exactly once
  (the reference's feature-column chunks re-read it D/offset times: ``chunking='columns'``).
* ``tn`` (reference :103-148): one batched GEMM producing all N partial blocks
  ``left[:, jR:(j+1)R]ᵀ·right`` into a contiguous send buffer (``left`` read transposed in
  place by the kernel's LDS transpose read), then ONE ``reduce_scatter`` — half the bytes and
  1/N the collective launches of the reference's N full all-reduces (with N-1 leaked
  handles).  Half-precision partials are reduced in fp32.
* No host barrier before each op (reference calls ``MPI.Barrier`` each time).
* ``schedule='ring'`` (or ``XDOT_OPS_SCHEDULE=ring``): the same three products as a ring of
  point-to-point hops (``Communicator.sendrecv``: RCCL ``batch_isend_irecv``): ``nt`` / ``all``
  pass each rank's ``right`` shard around the ring and consume the arriving shard with one
  GEMM while the next hop is in flight (two shard buffers instead of the gathered side);
  ``tn`` sends each destination's fp32 accumulator around the ring, every rank adding its
  partial (computed under the previous hop) — the reduce-scatter as N-1 hops.  Over xGMI's
  full mesh the collectives are faster (one link per hop vs all seven); the ring is the
  schedule whose resident comm buffers do not grow with N.

Output dtype = input dtype (the reference hard-codes fp32 via ``torch.empty`` without dtype
and therefore crashes in bf16); pass ``out_dtype=torch.float32`` for reference-identical fp32
outputs.  GPU tensors run on the HIP kernels; CPU tensors on torch.
"""
from __future__ import annotations

from typing import Optional

import torch

from ..ops import gemm as G
from ..utils import comm as _comm
from ..utils.checks import check_consistent
from ..utils.env import FLAGS
from ..utils.profiling import measure
from .schedule import (GROUP_BYTES, Offset, gather_pipeline, gather_rows_grouped, gather_rows_whole,
                       plan_chunks, resolve_offset)

__all__ = ["distributed_matmul_nt", "distributed_matmul_all", "distributed_matmul_tn",
           "distributed_matmul_block", "gather_sequence"]


def _prep(left: torch.Tensor, right: torch.Tensor, name: str):
    if left.shape[:-2] != right.shape[:-2]:
        raise ValueError(f"{name}: leading dims differ: {tuple(left.shape)} vs {tuple(right.shape)}")
    if left.device != right.device:
        raise ValueError(f"{name}: operands on different devices")


def _rmajor(x3: torch.Tensor) -> bool:
    """(Pn, R, D) view whose rows are R-major, i.e. the (1, H, R, d) head split of a contiguous
    (1, R, H*d) projection: gathered and produced in that layout, read by the GEMMs
    through their strides — no head-transpose or head-merge copy."""
    Pn, R, D = x3.shape
    return Pn > 1 and R > 1 and x3.stride() == (D, Pn * D, 1)


def _result_dtype(left, right, out_dtype):
    return out_dtype if out_dtype is not None else torch.promote_types(left.dtype, right.dtype)


@measure
def distributed_matmul_nt(left: torch.Tensor, right: torch.Tensor, offset: Offset = None, *,
                          comm: Optional[_comm.Communicator] = None, alpha: float = 1.0,
                          out_dtype: Optional[torch.dtype] = None, schedule: Optional[str] = None) -> torch.Tensor:
    """Row block ``r`` of ``L·Rᵀ``: (P, R, D) x (P, R, D) -> (P, R, T).

    ``offset``: rows of ``right`` gathered per step (``None``: whole shard; ``'auto'``:
    sized from free HBM).  Reference: ``functions.py:45-99``.
    """
    _prep(left, right, "distributed_matmul_nt")
    if left.shape[-1] != right.shape[-1]:
        raise ValueError("distributed_matmul_nt: feature dims differ")
    comm = comm or _comm.get_comm()
    n = comm.world_size
    P = tuple(left.shape[:-2])
    R, D = left.shape[-2], left.shape[-1]
    Rr = right.shape[-2]
    Pn = 1
    for d in P:
        Pn *= d
    T = Rr * n
    off = resolve_offset(offset, Rr, n * Pn * D * right.element_size(), right.device)
    chunks = plan_chunks(Rr, off)
    check_consistent(comm, "nt", left, right, tuple(chunks))
    out = torch.empty((Pn, R, T), dtype=_result_dtype(left, right, out_dtype), device=left.device)
    if R == 0 or T == 0:
        return out.view(*P, R, T)
    l3 = left.reshape(Pn, R, D)
    r3 = right.reshape(Pn, Rr, D)
    if _schedule(schedule) == "ring" and n > 1:
        _ring_nt(comm, l3, r3, out, alpha)
        return out.view(*P, R, T)

    def consume(s, e, gathered):  # gathered: (N, Pn, c, D)
        G.nt_chunk_into(out, l3, gathered, s, alpha)

    if len(chunks) > 1:  # offset-row all-gathers, grouped per GEMM (schedule.gather_rows_grouped)
        gather_rows_grouped(comm, r3, chunks, consume)
    elif _rmajor(r3) and n > 1:  # gather the (Rr, Pn*D) rows as they are; the GEMM reads them strided
        g = torch.empty((n, Rr, Pn, D), dtype=right.dtype, device=right.device)
        comm.all_gather_into(g, r3.transpose(0, 1))
        consume(0, Rr, g.permute(0, 2, 1, 3))
    else:
        gather_pipeline(comm, chunks, lambda s, e: r3[:, s:e, :], lambda c: (Pn, c, D), right.dtype,
                        right.device, consume)
    return out.view(*P, R, T)


@measure
def distributed_matmul_all(left: torch.Tensor, right: torch.Tensor, offset: Offset = None, *,
                           comm: Optional[_comm.Communicator] = None,
                           out_dtype: Optional[torch.dtype] = None, chunking: str = "rows",
                           schedule: Optional[str] = None) -> torch.Tensor:
    """Row block ``r`` of ``L·R``: (P, R, T) x (P, R, D) -> (P, R, D).

    ``offset`` bounds the per-step gather buffer exactly as in the reference, where a step
    gathers ``offset`` feature columns of every rank's ``right`` (N·R·offset elements;
    ``functions.py:161-212``).  ``chunking='columns'`` does literally that; each step then
    re-reads the whole (R, T) ``left`` block (D/offset passes: 32 at offset 24, D 768).  The
    default ``chunking='rows'`` spends the same buffer on ceil(R·offset/D) whole rows (all D
    features) of every rank per step and accumulates the K-partial products in fp32, so
    ``left`` is streamed exactly once whatever the offset.
    """
    _prep(left, right, "distributed_matmul_all")
    comm = comm or _comm.get_comm()
    n = comm.world_size
    P = tuple(left.shape[:-2])
    R, T = left.shape[-2], left.shape[-1]
    Rr, D = right.shape[-2], right.shape[-1]
    if T != Rr * n:
        raise ValueError(f"distributed_matmul_all: left has {T} columns, expected {Rr} x {n}")
    Pn = 1
    for d in P:
        Pn *= d
    if chunking not in ("rows", "columns"):
        raise ValueError(f"chunking must be 'rows' or 'columns', got {chunking!r}")
    off = resolve_offset(offset, D, n * Pn * Rr * right.element_size(), right.device)
    by_rows = chunking == "rows" and off is not None and off < D and Rr > 0
    if by_rows:  # same gather-buffer budget, whole rows: ceil(Rr * off / D) rows per step
        chunks = plan_chunks(Rr, max(1, -(-Rr * off // D)))
    else:
        chunks = plan_chunks(D, off)
    check_consistent(comm, "all", left, right, tuple(chunks))
    l3 = left.reshape(Pn, R, T)
    r3 = right.reshape(Pn, Rr, D)
    if _schedule(schedule) == "ring" and n > 1:
        out = torch.empty((Pn, R, D), dtype=_result_dtype(left, right, out_dtype), device=left.device)
        if R == 0 or D == 0:
            return out.reshape(*P, R, D)
        if T == 0:
            return out.zero_().reshape(*P, R, D)
        _ring_all(comm, l3, r3, out)
        return out.reshape(*P, R, D)
    rm = _rmajor(r3) and R > 1
    if rm:  # R-major like `right` (head-split view): the module's head merge is then a free view
        out = torch.empty((R, Pn, D), dtype=_result_dtype(left, right, out_dtype), device=left.device).transpose(0, 1)
    else:
        out = torch.empty((Pn, R, D), dtype=_result_dtype(left, right, out_dtype), device=left.device)
    if R == 0 or D == 0:
        return out.reshape(*P, R, D)
    if T == 0:
        return out.zero_().reshape(*P, R, D)

    if chunking == "rows" and Rr > 0 and n * Pn * Rr * D * right.element_size() <= 4 * GROUP_BYTES:
        # the whole gathered `right` fits the budget: every offset chunk still travels in its own
        # all-gather, then ONE K = T GEMM reads `left` whole (aligned rows, no per-rank K
        # segments starting off 16-byte boundaries when T/N is odd)
        G.matmul_into(out, l3, gather_rows_whole(comm, r3, chunks if by_rows else [(0, Rr)]))
        return out.reshape(*P, R, D)
    if by_rows:
        acc = out if out.dtype in (torch.float32, torch.float64) else torch.empty_like(out, dtype=torch.float32)

        def consume_rows(s, e, gathered):  # (N, Pn, c, D)
            G.all_rows_chunk_into(acc, l3, gathered, s, accumulate=s > 0)

        gather_rows_grouped(comm, r3, chunks, consume_rows)
        if acc is not out:
            out.copy_(acc)
        return out.reshape(*P, R, D)

    def consume(s, e, gathered):  # (N, Pn, Rr, c)
        G.all_chunk_into(out, l3, gathered, s)

    gather_pipeline(comm, chunks, lambda s, e: r3[..., s:e], lambda c: (Pn, Rr, c), right.dtype,
                    right.device, consume)
    return out.reshape(*P, R, D)


@measure
def distributed_matmul_tn(left: torch.Tensor, right: torch.Tensor, *,
                          comm: Optional[_comm.Communicator] = None,
                          out_dtype: Optional[torch.dtype] = None,
                          reduce_dtype: Optional[torch.dtype] = None, schedule: Optional[str] = None) -> torch.Tensor:
    """Row block ``r`` of ``Lᵀ·R``: (P, R, T) x (P, R, D) -> (P, R, D).

    One batched GEMM into an (N, P, R, D) send buffer + one reduce-scatter.
    Reference: ``functions.py:103-148``.
    """
    _prep(left, right, "distributed_matmul_tn")
    comm = comm or _comm.get_comm()
    n = comm.world_size
    P = tuple(left.shape[:-2])
    R, T = left.shape[-2], left.shape[-1]
    D = right.shape[-1]
    if right.shape[-2] != R:
        raise ValueError("distributed_matmul_tn: left/right row counts differ")
    if T % n != 0:
        raise ValueError(f"distributed_matmul_tn: {T} columns not divisible by world size {n}")
    Rc = T // n
    if Rc != R:
        raise ValueError("distributed_matmul_tn: column block size must equal the local row count")
    Pn = 1
    for d in P:
        Pn *= d
    check_consistent(comm, "tn", left, right)
    res_dt = _result_dtype(left, right, out_dtype)
    if reduce_dtype is None:
        reduce_dtype = torch.float32 if res_dt in (torch.bfloat16, torch.float16) and n > 1 else res_dt
    r3 = right.reshape(Pn, R, D)
    if _schedule(schedule) == "ring" and n > 1:
        if R == 0 or D == 0:
            return torch.zeros((*P, Rc, D), dtype=res_dt, device=left.device)
        return _ring_tn(comm, left.reshape(Pn, R, T), r3, reduce_dtype).to(res_dt).reshape(*P, Rc, D)
    rm = _rmajor(r3)  # R-major operand (head-split view) -> R-major send buffer and result
    if rm:
        sbuf = torch.empty((n, Rc, Pn, D), dtype=reduce_dtype, device=left.device)
        send = sbuf.permute(0, 2, 1, 3)
    else:
        sbuf = send = torch.empty((n, Pn, Rc, D), dtype=reduce_dtype, device=left.device)
    if R > 0 and D > 0:
        G.tn_partials_into(send, left.reshape(Pn, R, T), r3)
    else:
        sbuf.zero_()
    if n == 1:
        out = send[0]
    else:
        obuf = torch.empty(sbuf.shape[1:], dtype=reduce_dtype, device=left.device)
        comm.reduce_scatter(obuf, sbuf)
        out = obuf.transpose(0, 1) if rm else obuf
    return out.to(res_dt).reshape(*P, Rc, D)


# ---------------------------------------------------------------------------------------
# ring schedule (point-to-point hops)
# ---------------------------------------------------------------------------------------
def _schedule(schedule: Optional[str]) -> str:
    s = (schedule or FLAGS.ops_schedule or "gather").lower()
    if s not in ("gather", "ring"):
        raise ValueError(f"schedule must be 'gather' or 'ring', got {s!r}")
    return s


def _ring_pass(comm: _comm.Communicator, shard: torch.Tensor, consume) -> None:
    """Every rank's ``shard`` visits every rank: at step s rank r holds the shard of rank
    (r - s) mod N and calls ``consume(src, buf)`` on it while the hop of step s+1 is in flight.
    The rank's own shard is sent from the caller's tensor (never written); two receive buffers
    alternate.  Stream-ordered: a buffer is re-received into only after the hop that sent it
    completed and after the GEMM that read it was enqueued before that receive."""
    n, r = comm.world_size, comm.rank
    nxt, prv = (r + 1) % n, (r - 1) % n
    cur = shard.contiguous()
    spare = [torch.empty_like(cur), torch.empty_like(cur)]
    for s in range(n):
        h = None
        nb = None
        if s < n - 1:
            nb = spare[s % 2]
            h = comm.sendrecv(cur, nb, nxt, prv, async_op=True)
        consume((r - s) % n, cur)
        if h is not None:
            h.wait()
            cur = nb


def _ring_nt(comm, l3, r3, out, alpha):
    Rr = r3.shape[1]
    _ring_pass(comm, r3, lambda j, blk: G.nt_block_into(out[..., j * Rr:(j + 1) * Rr], l3, blk, alpha))


def _ring_all(comm, l3, r3, out):
    Rr = r3.shape[1]
    acc = out if out.dtype in (torch.float32, torch.float64) else torch.empty_like(out, dtype=torch.float32)
    first = [True]

    def consume(j, blk):
        G.all_rows_chunk_into(acc, l3, blk.unsqueeze(0), j * Rr, accumulate=not first[0])
        first[0] = False

    _ring_pass(comm, r3, consume)
    if acc is not out:
        out.copy_(acc)


def _ring_tn(comm, l3, r3, reduce_dtype):
    """Ring reduce-scatter of the tn partials: the accumulator of destination d starts at rank
    d+1 and travels N-1 hops, each rank adding left[:, :, d*R:(d+1)*R]ᵀ·right (computed while
    the previous hop is in flight); rank r ends holding destination r's sum."""
    n, r = comm.world_size, comm.rank
    Pn, R, D = r3.shape
    nxt, prv = (r + 1) % n, (r - 1) % n

    def partial(d, dst):
        G.tn_partials_into(dst.unsqueeze(0), l3[..., d * R:(d + 1) * R], r3)

    cur = torch.empty((Pn, R, D), dtype=reduce_dtype, device=r3.device)
    nb = torch.empty_like(cur)
    part = torch.empty_like(cur)
    partial((r - 1) % n, cur)
    for s in range(1, n):
        h = comm.sendrecv(cur, nb, nxt, prv, async_op=True)
        partial((r - 1 - s) % n, part)
        h.wait()
        nb.add_(part)
        cur, nb = nb, cur
    return cur


@measure
def distributed_matmul_block(left: torch.Tensor, right: torch.Tensor, transpose: bool = False, *,
                             comm: Optional[_comm.Communicator] = None) -> torch.Tensor:
    """``Σ_ranks left_r @ right_r`` (optionally transposed), Sum all-reduced.

    The reference's helper (``functions.py:151-157``) is dead code with two bugs — a
    ``.tranpose`` typo and Horovod's default *Average* op — this is the intended operation.
    """
    comm = comm or _comm.get_comm()
    block = G.matmul(left, right)
    if transpose:
        block = block.transpose(-1, -2).contiguous()
    comm.all_reduce(block, op="sum")
    return block


def gather_sequence(x: torch.Tensor, dim: int = -2, *, comm: Optional[_comm.Communicator] = None) -> torch.Tensor:
    """All-gather a sequence-sharded tensor along ``dim`` (rank-major), e.g. for inspection."""
    comm = comm or _comm.get_comm()
    n = comm.world_size
    if n == 1:
        return x
    dim = dim % x.dim()
    xm = x.movedim(dim, 0).contiguous()
    out = torch.empty((n,) + tuple(xm.shape), dtype=x.dtype, device=x.device)
    comm.all_gather_into(out, xm)
    out = out.reshape((n * xm.shape[0],) + tuple(xm.shape[1:]))
    return out.movedim(0, dim)
