"""Process-group façade: one process per GPU, ``torch.distributed`` over RCCL (xGMI) or gloo.

Replaces the reference's Horovod + mpi4py layer (reference:
``distributed_dot_product/utils/comm.py:1-30``: ``hvd.init()`` at import, ``get_world_size``
:13, ``get_rank`` :17, ``is_main_process`` :21, ``synchronize`` -> ``MPI.COMM_WORLD.Barrier``
:25-30).  Differences by design:

* nothing happens at import time; :func:`init` is called explicitly (or lazily by the first
  distributed op).  Rendezvous comes from the ``torchrun`` environment
  (``RANK``/``WORLD_SIZE``/``MASTER_ADDR``/``MASTER_PORT``); without it the job is a single
  rank and every collective is a local no-op/copy;
* ``backend='rccl'`` is accepted as an alias of torch's ``'nccl'`` (which *is* RCCL on ROCm);
* collectives are stream-ordered (``async_op=True`` returns a handle whose ``wait()`` makes
  the *current HIP stream* wait, never the host), so there are no fire-and-forget handles
  (reference quirk: ``functions.py:143-147`` leaks N-1 allreduce handles);
* :func:`synchronize` (host barrier) is kept for API parity but is never called on the hot
  path (the reference calls an MPI barrier before every op, ``functions.py:77,139,201``).

Three communicators implement one small protocol (:class:`Communicator`):

``TorchDistComm``  a ``torch.distributed`` process group (RCCL on GPU, gloo on CPU);
``LocalComm``      world size 1 — gathers are copies, reductions are identities;
``ThreadComm``     N logical ranks as N threads of one process (see :class:`ThreadGroup`),
                   used to exercise the exact multi-rank schedules and HIP kernels on a
                   single GPU and in CPU unit tests without spawning processes.
"""
from __future__ import annotations

import contextlib
import datetime
import os
import threading
from typing import List, Optional

import torch
import torch.distributed as dist

from .env import FLAGS

__all__ = [
    "Communicator", "TorchDistComm", "LocalComm", "EmulatedComm", "ThreadComm", "ThreadGroup", "Handle",
    "init", "is_initialized", "get_comm", "use_comm", "get_world_size", "get_rank",
    "get_local_rank", "is_main_process", "synchronize", "destroy", "resolve_backend", "check_collective_knobs",
]


class Handle:
    """Completion handle of an async collective.  ``wait()`` orders the caller's current
    stream after the collective (device-side for RCCL) and returns the output tensor."""

    __slots__ = ("_work", "_out", "_post")

    def __init__(self, work=None, out=None, post=None):
        self._work, self._out, self._post = work, out, post

    def wait(self):
        if self._work is not None:
            for w in (self._work if isinstance(self._work, (list, tuple)) else (self._work,)):
                w.wait()
            self._work = None
        if self._post is not None:
            self._post()
            self._post = None
        return self._out


class Communicator:
    """Minimal collective protocol used by every xdot schedule."""

    world_size: int = 1
    rank: int = 0
    # all_gather_into(out, out[rank]) (the input already in place in the output) is supported
    # without a staging copy of the own block
    inplace_gather: bool = False
    # all_reduce(op="avg") is one native collective (RCCL ncclAvg): the caller skips its division
    native_avg: bool = False

    # -- collectives ------------------------------------------------------------------
    def all_gather_into(self, out: torch.Tensor, inp: torch.Tensor, async_op: bool = False):
        """``out`` (contiguous, ``world_size * inp.numel()`` elements, rank-major) <- gather."""
        raise NotImplementedError

    def reduce_scatter(self, out: torch.Tensor, inp: torch.Tensor, async_op: bool = False):
        """``out`` <- sum over ranks of block ``rank`` of the rank-major ``inp``."""
        raise NotImplementedError

    def all_gather_chunks(self, raw: torch.Tensor, inp: torch.Tensor, sizes, async_op: bool = False):
        """``len(sizes)`` all-gathers issued together: chunk i = the next ``sizes[i]`` rows of the
        contiguous ``inp`` (rows, ...), gathered rank-major into the next ``N * sizes[i]`` rows'
        worth of the flat ``raw`` buffer (chunk i's output is (N, sizes[i], ...) contiguous).
        Every collective moves exactly its chunk (the reference's ``offset`` granularity);
        backends that can issue them as one grouped launch do (RCCL coalescing)."""
        hs = [self.all_gather_into(o, i, async_op=True) for o, i in _chunk_views(raw, inp, sizes, self.world_size)]
        h = Handle(out=raw, post=lambda: [x.wait() for x in hs if x is not None])
        if async_op:
            return h
        h.wait()
        return None

    def all_reduce(self, t: torch.Tensor, op: str = "sum", async_op: bool = False):
        raise NotImplementedError

    def all_reduce_multi(self, ts, op: str = "sum", async_op: bool = False):
        """``all_reduce`` of every tensor of ``ts`` in place, issued together (RCCL: one grouped
        launch), so a bucket of several gradients needs no flatten / copy-back passes."""
        hs = [self.all_reduce(t, op, async_op=True) for t in ts]
        h = Handle(out=ts, post=lambda: [x.wait() for x in hs if x is not None])
        if async_op:
            return h
        h.wait()
        return None

    def broadcast(self, t: torch.Tensor, src: int = 0, async_op: bool = False):
        raise NotImplementedError

    def all_gather_object(self, obj) -> list:
        raise NotImplementedError

    def barrier(self) -> None:
        raise NotImplementedError

    def sendrecv(self, send: torch.Tensor, recv: torch.Tensor, dst: int, src: int, async_op: bool = False):
        """Point-to-point exchange: ``send`` goes to rank ``dst`` while ``recv`` (same shape and
        dtype on every rank) is filled from rank ``src``.  Every rank of a ring calls it in the
        same order (one hop of :mod:`xdot.parallel.ring`)."""
        raise NotImplementedError

    def sendrecv_multi(self, pairs, async_op: bool = False):
        """Several point-to-point exchanges issued together: ``pairs`` = ``[(send, recv, dst,
        src), ...]``, each as :meth:`sendrecv`; backends that can run them as one group (one
        RCCL group: both directions of a bidirectional ring hop on two xGMI links at once) do."""
        hs = [self.sendrecv(s_, r_, d_, src_, async_op=True) for (s_, r_, d_, src_) in pairs]
        h = Handle(work=hs, out=[p[1] for p in pairs])
        if async_op:
            return h
        h.wait()
        return None

    @property
    def backend(self) -> str:
        return "local"

    def __repr__(self):
        return f"{type(self).__name__}(rank={self.rank}, world_size={self.world_size}, backend={self.backend})"


def _chunk_views(raw, inp, sizes, n):
    """(out_i (N, c_i, ...), in_i (c_i, ...)) of :meth:`Communicator.all_gather_chunks`."""
    rest = tuple(inp.shape[1:])
    row = 1
    for d in rest:
        row *= d
    views, off, r = [], 0, 0
    for c in sizes:
        views.append((raw[off:off + n * c * row].view((n, c) + rest), inp[r:r + c]))
        off += n * c * row
        r += c
    return views


def _runs(sizes):
    """consecutive equal sizes -> [(size, count)]"""
    out = []
    for c in sizes:
        if out and out[-1][0] == c:
            out[-1][1] += 1
        else:
            out.append([c, 1])
    return out


def _check_gather(out, inp, n):
    if out.numel() != inp.numel() * n:
        raise ValueError(f"all_gather_into: out has {out.numel()} elements, expected {n} x {inp.numel()}")
    if not out.is_contiguous():
        raise ValueError("all_gather_into: out must be contiguous")


class LocalComm(Communicator):
    """World size 1: the single-GPU degenerate case of every schedule."""

    world_size = 1
    rank = 0

    def all_gather_into(self, out, inp, async_op=False):
        _check_gather(out, inp, 1)
        if out.data_ptr() != inp.data_ptr():
            out.view(-1).copy_(inp.reshape(-1))
        return Handle(out=out) if async_op else None

    def reduce_scatter(self, out, inp, async_op=False):
        if out.data_ptr() != inp.data_ptr():
            out.view(-1).copy_(inp.reshape(-1))
        return Handle(out=out) if async_op else None

    def all_reduce(self, t, op="sum", async_op=False):
        return Handle(out=t) if async_op else None

    def broadcast(self, t, src=0, async_op=False):
        return Handle(out=t) if async_op else None

    def all_gather_object(self, obj):
        return [obj]

    def barrier(self):
        return None

    def sendrecv(self, send, recv, dst, src, async_op=False):
        # world size 1: the ring hop is to self (EmulatedComm: a device copy stands in for the link)
        if recv.data_ptr() != send.data_ptr():
            recv.copy_(send)
        return Handle(out=recv) if async_op else None


_LINK = {}


class EmulatedComm(LocalComm):
    """Rank ``rank`` of a pretend ``world_size``-rank job on ONE device (diagnostics only).

    Collectives keep their shapes and are replaced by device-local copies (the gather
    replicates the local shard, the reduce-scatter takes this rank's slice) so a single GPU
    runs exactly the per-rank compute of an N-GPU step, without the transport.  Used by
    ``benchmarks/bench_rank.py`` to study the N=8 per-rank step on the one-GPU box; never
    by tests of numerical results (the math of an emulated job is not a real N-rank job).

    Link model (``link_gbps`` set, GPU tensors): every collective runs on its own "link"
    stream, ordered after the caller's stream, as a spin of ``bytes on the wire / rate``
    followed by the copy; ``Handle.wait()`` orders the waiting stream after it.  So the
    one-GPU timeline shows what overlaps a transfer of that length and what waits for it —
    the async stream discipline of the RCCL path (a collective's stream, events, recycled
    buffers) is exercised for real.  Bytes on the wire per rank: all-gather and
    reduce-scatter ``(N-1)/N`` of the full buffer, all-reduce twice that, at ``link_gbps``
    (an all-gather bus bandwidth); a ring hop ``send.nbytes`` at ``p2p_gbps`` (one xGMI link).
    """

    def __init__(self, world_size: int, rank: int = 0, link_gbps: Optional[float] = None,
                 p2p_gbps: Optional[float] = None):
        self.world_size, self.rank = int(world_size), int(rank)
        self.link_gbps = link_gbps
        self.p2p_gbps = p2p_gbps or link_gbps
        self._cycles_per_s = None

    @property
    def backend(self):
        return "emulated"

    def _spin_cycles(self, seconds: float, dev) -> int:
        if self._cycles_per_s is None:  # calibrate torch.cuda._sleep's counter once
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda._sleep(1000)
            s.record()
            torch.cuda._sleep(2_000_000)
            e.record()
            e.synchronize()
            self._cycles_per_s = 2_000_000 / (s.elapsed_time(e) * 1e-3)
        return int(seconds * self._cycles_per_s)

    def _transfer(self, out, nbytes, rate_gbps, fn, async_op, keep=()):
        if rate_gbps is None or not out.is_cuda:
            fn()
            return Handle(out=out) if async_op else None
        dev = out.device
        cur = torch.cuda.current_stream(dev)
        link = _LINK.get(dev)
        if link is None:
            # one high-priority link stream per device for every emulated communicator (as RCCL's
            # TORCH_NCCL_HIGH_PRIORITY streams): each extra stream takes a hardware queue
            # (GPU_MAX_HW_QUEUES = 4), and past that streams share queues and serialise
            link = _LINK[dev] = torch.cuda.Stream(device=dev, priority=-1)
        link.wait_stream(cur)
        with torch.cuda.stream(link):
            cyc = self._spin_cycles(nbytes / (rate_gbps * 1e9), dev)
            if cyc > 0:
                torch.cuda._sleep(cyc)
            fn()
            ev = torch.cuda.Event()
            ev.record(link)
        for t in (out,) + tuple(keep):
            t.record_stream(link)
        h = Handle(out=out, post=lambda: torch.cuda.current_stream(dev).wait_event(ev))
        if async_op:
            return h
        h.wait()
        return None

    inplace_gather = True
    native_avg = True  # (the modelled all-reduce moves the same bytes for sum and avg)

    def all_gather_into(self, out, inp, async_op=False):
        _check_gather(out, inp, self.world_size)
        n, r = self.world_size, self.rank

        def fill():
            ov, src = out.view(n, -1), inp.reshape(1, -1)
            if inp.data_ptr() == ov[r].data_ptr():  # in place: replicate into the other blocks only
                if r > 0:
                    ov[:r].copy_(src.expand(r, -1))
                if r < n - 1:
                    ov[r + 1:].copy_(src.expand(n - r - 1, -1))
            else:
                ov.copy_(src.expand(n, -1))
        return self._transfer(out, out.nbytes * (n - 1) // n, self.link_gbps, fill, async_op, (inp,))

    def all_gather_chunks(self, raw, inp, sizes, async_op=False):
        n = self.world_size
        row = inp[0].numel() if inp.shape[0] else 0

        def copy():  # one replicate copy per run of equal-size chunks
            off = r = 0
            for c, cnt in _runs(sizes):
                src = inp[r:r + c * cnt].reshape(cnt, 1, c * row)
                raw[off:off + cnt * n * c * row].view(cnt, n, c * row).copy_(src.expand(cnt, n, c * row))
                off += cnt * n * c * row
                r += c * cnt
        used = raw[:n * sum(sizes) * row]
        return self._transfer(used, used.nbytes * (n - 1) // n, self.link_gbps, copy, async_op, (inp,))

    def reduce_scatter(self, out, inp, async_op=False):
        n = self.world_size
        return self._transfer(out, inp.nbytes * (n - 1) // n, self.link_gbps,
                              lambda: out.view(-1).copy_(inp.reshape(n, -1)[self.rank]), async_op, (inp,))

    def all_reduce(self, t, op="sum", async_op=False):
        n = self.world_size
        return self._transfer(t, 2 * t.nbytes * (n - 1) // n, self.link_gbps, lambda: None, async_op)

    def sendrecv(self, send, recv, dst, src, async_op=False):
        def hop():
            if recv.data_ptr() != send.data_ptr():
                recv.copy_(send)
        return self._transfer(recv, send.nbytes, self.p2p_gbps, hop, async_op, (send,))

    def sendrecv_multi(self, pairs, async_op=False):
        # the exchanges go to different peers (different xGMI links): one transfer as long as
        # the largest of them
        def hops():
            for s_, r_, _d, _s in pairs:
                if r_.data_ptr() != s_.data_ptr():
                    r_.copy_(s_)
        nbytes = max(p[0].nbytes for p in pairs)
        keep = tuple(p[0] for p in pairs) + tuple(p[1] for p in pairs[1:])
        h = self._transfer(pairs[0][1], nbytes, self.p2p_gbps, hops, True, keep)
        h._out = [p[1] for p in pairs]
        if async_op:
            return h
        h.wait()
        return None

    def all_gather_object(self, obj):
        return [obj] * self.world_size


_OPS = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN,
        "avg": dist.ReduceOp.AVG if hasattr(dist.ReduceOp, "AVG") else None}


class TorchDistComm(Communicator):
    """A ``torch.distributed`` process group.  On GPU the backend is RCCL over xGMI."""

    def __init__(self, group=None):
        self.group = group
        self.world_size = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self._backend = dist.get_backend(group)

    @property
    def backend(self):
        return str(self._backend)

    def _staged(self, *ts) -> bool:
        """gloo cannot run these collectives on device memory: stage GPU tensors through the
        host (used to emulate several ranks on one GPU in tests; never on the RCCL path)."""
        return self._backend == "gloo" and any(t.is_cuda for t in ts)

    @property
    def inplace_gather(self) -> bool:
        return self._backend == "nccl"  # RCCL all-gather in place: sendbuff = recvbuff + rank block

    @property
    def native_avg(self) -> bool:
        return self._backend == "nccl" and _OPS["avg"] is not None  # gloo has no AVG

    def all_gather_into(self, out, inp, async_op=False):
        _check_gather(out, inp, self.world_size)
        if self._backend != "nccl" and inp.data_ptr() == out.view(self.world_size, -1)[self.rank].data_ptr():
            inp = inp.clone()  # gloo: no aliasing between the input and the output
        if self._staged(out, inp):
            o = torch.empty(out.shape, dtype=out.dtype)
            self.all_gather_into(o, inp.detach().cpu())
            out.copy_(o)
            return Handle(out=out) if async_op else None
        inp = inp.contiguous()
        w = dist.all_gather_into_tensor(out.view(-1), inp.view(-1), group=self.group, async_op=async_op)
        return Handle(w, out) if async_op else None

    def all_reduce_multi(self, ts, op="sum", async_op=False):
        if self._backend != "nccl" or len(ts) < 2 or not hasattr(dist, "_coalescing_manager") or \
                any(self._staged(t) for t in ts):
            return super().all_reduce_multi(ts, op, async_op)
        # one grouped RCCL launch, every tensor reduced in place
        with dist._coalescing_manager(group=self.group, device=ts[0].device, async_ops=True) as cm:
            for t in ts:
                dist.all_reduce(t, op=_OPS[op], group=self.group)
        h = Handle(cm, ts)
        if async_op:
            return h
        h.wait()
        return None

    def all_gather_chunks(self, raw, inp, sizes, async_op=False):
        views = _chunk_views(raw, inp, sizes, self.world_size)
        if self._backend != "nccl" or len(views) < 2 or not hasattr(dist, "_coalescing_manager"):
            return super().all_gather_chunks(raw, inp, sizes, async_op)
        # one grouped RCCL launch for every chunk's all-gather
        with dist._coalescing_manager(group=self.group, device=raw.device, async_ops=True) as cm:
            for o, i in views:
                dist.all_gather_into_tensor(o.view(-1), i.contiguous().view(-1), group=self.group)
        h = Handle(cm, raw)
        if async_op:
            return h
        h.wait()
        return None

    def reduce_scatter(self, out, inp, async_op=False):
        if inp.numel() != out.numel() * self.world_size:
            raise ValueError("reduce_scatter: size mismatch")
        if self._staged(out, inp):
            o = torch.empty(out.shape, dtype=out.dtype)
            self.reduce_scatter(o, inp.detach().cpu())
            out.copy_(o)
            return Handle(out=out) if async_op else None
        inp = inp.contiguous()
        if self._backend == "gloo" and inp.dtype in (torch.bfloat16, torch.float16):
            # reduce in fp32 on gloo (no half reductions on CPU backends)
            tmp = torch.empty(out.numel(), dtype=torch.float32, device=out.device)
            w = dist.reduce_scatter_tensor(tmp, inp.view(-1).float(), group=self.group, async_op=async_op)
            post = lambda: out.view(-1).copy_(tmp)  # noqa: E731
            if async_op:
                return Handle(w, out, post)
            post()
            return None
        o = out if out.is_contiguous() else torch.empty_like(out, memory_format=torch.contiguous_format)
        w = dist.reduce_scatter_tensor(o.view(-1), inp.view(-1), group=self.group, async_op=async_op)
        post = None if o is out else (lambda: out.copy_(o))
        if async_op:
            return Handle(w, out, post)
        if post:
            post()
        return None

    def all_reduce(self, t, op="sum", async_op=False):
        if self._staged(t):
            c = t.detach().cpu()
            dist.all_reduce(c, op=_OPS[op], group=self.group)
            t.copy_(c)
            return Handle(out=t) if async_op else None
        w = dist.all_reduce(t, op=_OPS[op], group=self.group, async_op=async_op)
        return Handle(w, t) if async_op else None

    def broadcast(self, t, src=0, async_op=False):
        if self._staged(t):
            c = t.detach().cpu()
            dist.broadcast(c, src=src, group=self.group)
            t.copy_(c)
            return Handle(out=t) if async_op else None
        w = dist.broadcast(t, src=src, group=self.group, async_op=async_op)
        return Handle(w, t) if async_op else None

    def all_gather_object(self, obj):
        res = [None] * self.world_size
        dist.all_gather_object(res, obj, group=self.group)
        return res

    def barrier(self):
        dist.barrier(group=self.group)

    def _global(self, r: int) -> int:
        return r if self.group is None else dist.get_global_rank(self.group, r)

    def sendrecv(self, send, recv, dst, src, async_op=False):
        if self._staged(send, recv):
            c = torch.empty(recv.shape, dtype=recv.dtype)
            self.sendrecv(send.detach().cpu().contiguous(), c, dst, src)
            recv.copy_(c)
            return Handle(out=recv) if async_op else None
        send = send.contiguous()
        if self._backend == "nccl":
            # one RCCL group: the send and the receive of a ring hop progress together on the
            # collective stream; wait() orders the caller's stream after both
            works = dist.batch_isend_irecv([dist.P2POp(dist.isend, send, self._global(dst), self.group),
                                            dist.P2POp(dist.irecv, recv, self._global(src), self.group)])
        else:
            works = [dist.isend(send, self._global(dst), group=self.group),
                     dist.irecv(recv, self._global(src), group=self.group)]
        h = Handle(list(works), recv)
        if async_op:
            return h
        h.wait()
        return None

    def sendrecv_multi(self, pairs, async_op=False):
        if self._backend != "nccl" or any(self._staged(p[0], p[1]) for p in pairs):
            return super().sendrecv_multi(pairs, async_op)
        ops = []
        for s_, r_, d_, src_ in pairs:  # ONE RCCL group: every send / receive progresses together
            ops.append(dist.P2POp(dist.isend, s_.contiguous(), self._global(d_), self.group))
            ops.append(dist.P2POp(dist.irecv, r_, self._global(src_), self.group))
        h = Handle(list(dist.batch_isend_irecv(ops)), [p[1] for p in pairs])
        if async_op:
            return h
        h.wait()
        return None


# ----------------------------------------------------------------------------------------
# ThreadComm: N logical ranks inside one process (emulated multi-rank on one device)
# ----------------------------------------------------------------------------------------
class ThreadGroup:
    """Shared state of N emulated ranks.  Each rank runs in its own Python thread and talks
    through :meth:`comm`.  Device work is ordered with events, so the collectives are
    stream-correct on a GPU (each thread may use its own stream)."""

    def __init__(self, world_size: int, timeout: float = 120.0, ring_reduce: bool = False):
        """``ring_reduce``: reduce-scatter 16-bit tensors the way RCCL's ring does -- in the
        tensor's own dtype, one rounding per hop, block r accumulated from rank r+1 around to
        rank r -- instead of gloo's fp32 accumulation (numerics tests of the default bf16
        gradient partials)."""
        self.world_size = world_size
        self.ring_reduce = ring_reduce
        self._barrier = threading.Barrier(world_size, timeout=timeout)
        self._slots: List[object] = [None] * world_size

    def comm(self, rank: int) -> "ThreadComm":
        return ThreadComm(self, rank)

    def run(self, fn, *args, **kwargs):
        """Run ``fn(rank, *args, **kwargs)`` on every rank (one thread each) with that rank's
        communicator installed as the default; returns the per-rank results."""
        results: List[object] = [None] * self.world_size
        errors: List[BaseException] = []

        def body(r):
            try:
                with use_comm(self.comm(r)):
                    results[r] = fn(r, *args, **kwargs)
            except BaseException as e:  # noqa: BLE001
                errors.append(e)
                self._barrier.abort()

        threads = [threading.Thread(target=body, args=(r,), daemon=True) for r in range(self.world_size)]
        for t in threads:
            t.start()
        for t in threads:
            t.join()
        if errors:
            real = [e for e in errors if not isinstance(e, threading.BrokenBarrierError)]
            raise (real or errors)[0]
        return results


class ThreadComm(Communicator):
    def __init__(self, group: ThreadGroup, rank: int):
        self.g = group
        self.world_size = group.world_size
        self.rank = rank

    @property
    def backend(self):
        return "thread"

    def _exchange(self, value):
        """Publish ``value``; return every rank's value.  Device tensors are published with an
        event so consumers order their own streams after the producer's writes."""
        ev = None
        if isinstance(value, torch.Tensor) and value.is_cuda:
            ev = torch.cuda.Event()
            ev.record()
        self.g._slots[self.rank] = (value, ev)
        self.g._barrier.wait()
        vals = list(self.g._slots)
        self.g._barrier.wait()
        out = []
        for v, e in vals:
            if e is not None:
                torch.cuda.current_stream().wait_event(e)
            out.append(v)
        return out

    def _done(self, t):
        """Second phase: hold peers until every rank finished reading published tensors."""
        if isinstance(t, torch.Tensor) and t.is_cuda:
            torch.cuda.current_stream().synchronize()
        self.g._barrier.wait()

    def all_gather_into(self, out, inp, async_op=False):
        _check_gather(out, inp, self.world_size)
        parts = self._exchange(inp.contiguous())
        ov = out.view(self.world_size, -1)
        for r, p in enumerate(parts):
            ov[r].copy_(p.reshape(-1))
        self._done(out)
        return Handle(out=out) if async_op else None

    def reduce_scatter(self, out, inp, async_op=False):
        parts = self._exchange(inp.contiguous())
        n = out.numel()
        if self.g.ring_reduce and out.dtype in (torch.bfloat16, torch.float16):
            ws = self.world_size
            blk = [p.reshape(-1)[self.rank * n:(self.rank + 1) * n] for p in parts]
            acc = blk[(self.rank + 1) % ws].clone()
            for s in range(2, ws + 1):  # one rounding to the wire dtype per ring hop
                acc = (acc.float() + blk[(self.rank + s) % ws].float()).to(out.dtype)
            out.view(-1).copy_(acc) if out.is_contiguous() else out.copy_(acc.view(out.shape))
            self._done(out)
            return Handle(out=out) if async_op else None
        acc_dt = torch.float32 if out.dtype in (torch.bfloat16, torch.float16) else out.dtype
        acc = torch.zeros(n, dtype=acc_dt, device=out.device)
        for p in parts:
            acc += p.reshape(-1)[self.rank * n:(self.rank + 1) * n].to(acc.dtype)
        out.view(-1).copy_(acc) if out.is_contiguous() else out.copy_(acc.view(out.shape))
        self._done(out)
        return Handle(out=out) if async_op else None

    def all_reduce(self, t, op="sum", async_op=False):
        parts = self._exchange(t.clone())
        res = parts[0].clone()
        for p in parts[1:]:
            if op == "sum":
                res += p
            elif op == "max":
                res = torch.maximum(res, p)
            elif op == "min":
                res = torch.minimum(res, p)
            elif op == "avg":
                res += p
            else:
                raise ValueError(op)
        if op == "avg":
            res /= len(parts)
        t.copy_(res)
        self._done(t)
        return Handle(out=t) if async_op else None

    def broadcast(self, t, src=0, async_op=False):
        parts = self._exchange(t.clone() if self.rank == src else None)
        t.copy_(parts[src])
        self._done(t)
        return Handle(out=t) if async_op else None

    def all_gather_object(self, obj):
        return self._exchange(obj)

    def barrier(self):
        self.g._barrier.wait()

    def sendrecv(self, send, recv, dst, src, async_op=False):
        parts = self._exchange(send.contiguous())
        recv.copy_(parts[src])
        self._done(recv)
        return Handle(out=recv) if async_op else None


# ----------------------------------------------------------------------------------------
# default communicator management
# ----------------------------------------------------------------------------------------
_DEFAULT: Optional[Communicator] = None
_LOCAL = threading.local()


def resolve_backend(backend: str = "auto") -> str:
    b = (backend or "auto").lower()
    if b in ("rccl", "nccl"):
        return "nccl"
    if b == "gloo":
        return "gloo"
    if b == "auto":
        return "nccl" if torch.cuda.is_available() else "gloo"
    raise ValueError(f"unknown backend {backend!r} (expected auto|rccl|nccl|gloo)")


def get_local_rank() -> int:
    return int(os.environ.get("LOCAL_RANK", os.environ.get("RANK", "0")))


def init(backend: str = "auto", timeout_s: Optional[float] = None, set_device: bool = True) -> Communicator:
    """Initialise (idempotently) the default communicator from the torchrun environment.

    ``backend``: ``'auto'`` (RCCL if a GPU is visible, else gloo), ``'rccl'``/``'nccl'``, ``'gloo'``.
    ``timeout_s`` bounds every collective so a rank mismatch surfaces as an error rather than
    a hang (reference: no timeouts at all).
    """
    global _DEFAULT
    if _DEFAULT is not None:
        return _DEFAULT
    if dist.is_available() and dist.is_initialized():
        _DEFAULT = TorchDistComm()
        return _DEFAULT
    if "WORLD_SIZE" not in os.environ or "MASTER_ADDR" not in os.environ:
        _DEFAULT = LocalComm()  # plain `python script.py`: one rank, no process group
        return _DEFAULT
    be = resolve_backend(backend)
    if be == "nccl":
        os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
        # RCCL's kernels share the CUs with long-running attention kernels: high-priority
        # collective streams let their workgroups dispatch as soon as any slot frees
        os.environ.setdefault("TORCH_NCCL_HIGH_PRIORITY", "1")
        if set_device and torch.cuda.is_available():
            torch.cuda.set_device(get_local_rank() % max(1, torch.cuda.device_count()))
    kw = {}
    t = timeout_s if timeout_s is not None else FLAGS.comm_timeout_s
    kw["timeout"] = datetime.timedelta(seconds=t)
    if be == "nccl" and torch.cuda.is_available():
        kw["device_id"] = torch.device("cuda", torch.cuda.current_device())
    dist.init_process_group(be, **kw)
    _DEFAULT = TorchDistComm()
    check_collective_knobs(_DEFAULT)
    if _DEFAULT.world_size > 1 and torch.cuda.is_available() and FLAGS.ipc:
        # stage 2: xGMI pull all-gather / reduce-scatter (csrc/ipc.hip).  Over gloo too: several
        # ranks sharing one GPU rehearse the device-side collectives (RCCL refuses that layout)
        from .ipc import IpcComm
        if be == "gloo":
            torch.cuda.set_device(get_local_rank() % max(1, torch.cuda.device_count()) if set_device else 0)
        _DEFAULT = IpcComm(_DEFAULT)
    return _DEFAULT


def check_collective_knobs(comm: "Communicator") -> None:
    """Raise on every rank if the ranks disagree on a flag that changes the number or dtype
    of the collectives an op issues (``xdot.utils.env.COLLECTIVE_KNOBS``: gather chunks,
    local-first, IPC, ops schedule, ...).  Mismatched ranks would otherwise issue different
    collective sequences and hang until the timeout.  Called by :func:`init` for multi-rank
    communicators (the reference asserts its world size at init: ``utils/comm.py:8-9``)."""
    if comm.world_size == 1:
        return
    from .env import collective_knobs

    mine = collective_knobs()
    everyone = comm.all_gather_object(mine)
    bad = sorted(k for k in mine if any(o.get(k) != mine[k] for o in everyone))
    if bad:
        vals = {k: [o.get(k) for o in everyone] for k in bad}
        raise RuntimeError(f"xdot: ranks disagree on collective-shaping flags {vals} (per rank); set the same "
                           "XDOT_* environment on every rank")


def is_initialized() -> bool:
    return _DEFAULT is not None or getattr(_LOCAL, "comm", None) is not None


def destroy() -> None:
    global _DEFAULT
    if hasattr(_DEFAULT, "close"):
        _DEFAULT.close()
    if isinstance(getattr(_DEFAULT, "base", _DEFAULT), TorchDistComm) and dist.is_initialized():
        dist.destroy_process_group()
    _DEFAULT = None


def get_comm() -> Communicator:
    c = getattr(_LOCAL, "comm", None)
    if c is not None:
        return c
    return _DEFAULT if _DEFAULT is not None else init()


@contextlib.contextmanager
def use_comm(c: Communicator):
    """Install ``c`` as the default communicator of the current thread."""
    prev = getattr(_LOCAL, "comm", None)
    _LOCAL.comm = c
    try:
        yield c
    finally:
        _LOCAL.comm = prev


def get_world_size() -> int:
    """reference: ``utils/comm.py:13``"""
    return get_comm().world_size


def get_rank() -> int:
    """reference: ``utils/comm.py:17``"""
    return get_comm().rank


def is_main_process() -> bool:
    """reference: ``utils/comm.py:21``"""
    return get_rank() == 0


def synchronize() -> None:
    """Host barrier across ranks (reference: ``utils/comm.py:25-30``).  Off the hot path."""
    get_comm().barrier()
