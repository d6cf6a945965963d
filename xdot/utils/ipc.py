"""Native xGMI pull collectives over HIP IPC (SURVEY §5.8 stage 2, ``csrc/ipc.hip``).

:class:`IpcComm` wraps a ``torch.distributed`` communicator (one process per GPU of a node)
and replaces its two bulk data movers — the ones the attention and the distributed products
spend their bytes in (reference: ``multiplication/functions.py:89-97`` gather loop and the
N all-reduces at ``:143-147``, ``:202-210``) — with one kernel each that reads the peers'
memory directly over the point-to-point xGMI links:

* ``all_gather_into``: every rank stages its shard in an IPC-exported buffer; every rank pulls
  the N-1 peer shards concurrently (its workgroups start at different peers, so all 7 links of
  an MI355X carry traffic at once instead of one ring hop per step);
* ``reduce_scatter``: every rank pulls its own block from each peer and sums the N blocks in
  fp32 in rank order 0..N-1 — deterministic and rounded once to the output dtype (RCCL's ring
  rounds bf16 partials after every hop: ``tests/test_bf16_reduce.py``).

Everything else (all-reduce, broadcast, p2p, object gathers, barriers) and every call the pull
kernels do not cover (1-byte dtypes, blocks that are not a multiple of 16 bytes, messages
beyond the staging capacity, CPU tensors) goes to the wrapped communicator.  Those decisions
depend only on shapes and dtypes, so every rank takes the same route.

Synchronisation is device-side (per (peer, byte-range) epoch flags in uncached signal pages);
the host never blocks.  The pull kernels run on a dedicated high-priority communication
stream (ordered after the caller's stream for their inputs) and ``async_op=True`` returns an
event-backed :class:`~xdot.utils.comm.Handle`: the caller's stream keeps computing (e.g. the
attention's local block) while the pull runs, and ``Handle.wait()`` orders it after the kernel.
Every device wait is bounded (``XDOT_IPC_TIMEOUT_S``, default: the process-group timeout
``XDOT_COMM_TIMEOUT_S``, 600 s, so a peer busy with host work such as checkpointing is not
mistaken for a dead one): on expiry the kernel writes NaN over the output range that peer
should have supplied (the result is unusable), sets a host-mapped error word and drains; the
host raises at the next collective (``Handle.wait()`` raises for earlier collectives, and for
its own one only under ``XDOT_CHECK=1``, which synchronises on the kernel first).

Enable with ``XDOT_IPC=1`` (``xdot.utils.comm.init`` wraps its RCCL communicator) or build one
explicitly: ``IpcComm(comm)``.  The staging buffers hold ``XDOT_IPC_MB`` MiB per slot (two
slots per rank, default 512 MiB: the bf16 ``[q|v]`` shard of a T=200000 rank at N=8 is 77 MB).
"""
from __future__ import annotations

import os
from typing import List, Optional

import torch

from .. import _ext
from .comm import Communicator, Handle, _check_gather
from .env import FLAGS

__all__ = ["IpcComm", "ipc_available"]


def ipc_available() -> bool:
    return torch.cuda.is_available() and _ext.load() and hasattr(torch.ops.xdot, "ipc_all_gather")


class IpcError(RuntimeError):
    pass


class _EventWork:
    """``wait()`` orders the caller's current stream after a recorded event (device-side)."""

    __slots__ = ("ev", "device")

    def __init__(self, ev, device):
        self.ev = ev
        self.device = device

    def wait(self):
        torch.cuda.current_stream(self.device).wait_event(self.ev)

    def is_completed(self) -> bool:
        return self.ev.query()


class IpcComm(Communicator):
    """Pull-based all-gather / reduce-scatter over IPC-mapped peer memory; the rest delegates
    to ``base`` (which also exchanges the IPC handles)."""

    def __init__(self, base: Communicator, capacity_mb: Optional[float] = None,
                 timeout_s: Optional[float] = None, nwg: Optional[int] = None, device=None):
        if not ipc_available():
            raise IpcError("IpcComm needs a GPU and the xdot extension")
        ops = torch.ops.xdot
        sig_bytes, max_ranks, max_wgs, _hb, khz = ops.ipc_info()
        self.base = base
        self.world_size, self.rank = base.world_size, base.rank
        if not 2 <= self.world_size <= max_ranks:
            raise IpcError(f"IpcComm: world size {self.world_size} outside 2..{max_ranks} (one node)")
        self.device = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
        cap = float(capacity_mb if capacity_mb is not None else FLAGS.ipc_mb)
        self.capacity = (int(cap * 2**20) + 255) // 256 * 256
        t = float(timeout_s if timeout_s is not None else FLAGS.ipc_timeout_s)
        self.ticks = int(t * khz * 1000) if khz > 0 else int(t * 1e8)
        self.max_wgs = int(max_wgs)
        w = int(nwg if nwg is not None else FLAGS.ipc_wgs)
        self.nwg = max(1, min(self.max_wgs, w))  # byte ranges = workgroups per collective
        self.epoch = 0
        self._stream = None  # high-priority communication stream (created on first use)
        with torch.cuda.device(self.device):
            self._stage = ops.ipc_alloc(2 * self.capacity, False)
            self._sig = ops.ipc_alloc(int(sig_bytes), True)
            self._host, self._status = ops.ipc_host_word()
            mine = (ops.ipc_get_handle(self._stage).tolist(), ops.ipc_get_handle(self._sig).tolist(),
                    os.getpid(), self.capacity, self.nwg)
            allh = base.all_gather_object(mine)
            # routing (IPC vs the wrapped communicator) and the peers' stage offsets follow from
            # the capacity, the flag partition from nwg: ranks that disagree would hang or read
            # past a peer's staging allocation
            shapes = {(c, w) for (_hs, _hg, _pid, c, w) in allh}
            if len(shapes) != 1:
                ops.ipc_free(self._stage)
                ops.ipc_free(self._sig)
                raise IpcError(f"IpcComm: ranks disagree on (staging bytes, workgroups): {sorted(shapes)} "
                               f"(XDOT_IPC_MB / XDOT_IPC_WGS must match on every rank)")
            self._opened: List[int] = []
            self.stage_ptrs, self.sig_ptrs = [], []
            for p, (hs, hg, _pid, _c, _w) in enumerate(allh):
                if p == self.rank:
                    self.stage_ptrs.append(self._stage)
                    self.sig_ptrs.append(self._sig)
                    continue
                s = ops.ipc_open(torch.tensor(hs, dtype=torch.uint8))
                g = ops.ipc_open(torch.tensor(hg, dtype=torch.uint8))
                self._opened += [s, g]
                self.stage_ptrs.append(s)
                self.sig_ptrs.append(g)
        base.barrier()  # every rank mapped every page before the first pull

    inplace_gather = True  # the pull kernel skips the own-block copy when inp is out[rank]

    @property
    def native_avg(self) -> bool:  # all-reduce is the base communicator's
        return self.base.native_avg

    @property
    def backend(self) -> str:
        return f"ipc+{self.base.backend}"

    # -- routing ------------------------------------------------------------------------
    def _pullable(self, *ts: torch.Tensor, stage_bytes: int) -> bool:
        # not under HIP-graph capture: the epoch is a host counter baked into the launch, a
        # replay would reuse it (the wrapped RCCL collectives are capturable)
        return (all(t.is_cuda for t in ts) and all(t.element_size() >= 2 for t in ts)
                and 0 < stage_bytes <= self.capacity and not torch.cuda.is_current_stream_capturing())

    def _wgs(self, shard_bytes: int) -> int:
        # ONE partition for every collective of this communicator: the (peer, range) flags of
        # epoch e are checked against those of e - 2, so the range count must never change
        return self.nwg

    def check(self) -> None:
        """Raise if a device-side wait of an earlier collective timed out (a peer stopped)."""
        if torch.ops.xdot.ipc_read_word(self._host):
            raise IpcError(f"rank {self.rank}: an xGMI pull collective timed out waiting for a peer "
                           f"(XDOT_IPC_TIMEOUT_S); its output is invalid")

    def _post(self, ev) -> None:
        """After ``Handle.wait()``: a timeout of THIS collective is only known once its kernel has
        finished, so it surfaces at the next collective (``_next``) or, under ``XDOT_CHECK=1``,
        here after synchronising on the kernel; earlier timeouts raise here either way."""
        if FLAGS.check:
            ev.synchronize()
        self.check()

    def _next(self):
        self.check()
        self.epoch += 1
        off = (self.epoch & 1) * self.capacity
        return [p + off for p in self.stage_ptrs]

    def _launch(self, fn, out, tensors, async_op):
        """Run ``fn()`` (one pull kernel) on the communication stream, ordered after the
        caller's stream; returns an event-backed Handle (async) or orders the caller's stream
        after the kernel (sync; the host never blocks either way)."""
        cur = torch.cuda.current_stream(self.device)
        if self._stream is None:
            self._stream = torch.cuda.Stream(device=self.device, priority=-1)
        cs = self._stream
        cs.wait_stream(cur)
        with torch.cuda.stream(cs):
            fn()
        ev = torch.cuda.Event()
        ev.record(cs)
        for t in tensors:  # the caching allocator must not recycle them while the kernel runs
            t.record_stream(cs)
        if async_op:
            return Handle(work=_EventWork(ev, self.device), out=out, post=lambda: self._post(ev))
        cur.wait_event(ev)
        return None

    # -- pull collectives ---------------------------------------------------------------
    def all_gather_into(self, out, inp, async_op=False):
        _check_gather(out, inp, self.world_size)
        nb = inp.numel() * inp.element_size()
        if not (self._pullable(out, inp, stage_bytes=nb) and nb % 16 == 0):
            return self.base.all_gather_into(out, inp, async_op)
        if not out.is_contiguous():  # same on every rank (layout follows the shapes)
            return self.base.all_gather_into(out, inp, async_op)
        i = inp.contiguous()
        stage = self._next()
        ep, wgs = self.epoch, self._wgs(nb)
        return self._launch(lambda: torch.ops.xdot.ipc_all_gather(i, out.view(-1), stage, self.sig_ptrs, self._status,
                                                                  self.rank, ep, self.ticks, wgs),
                            out, (i, out), async_op)

    def reduce_scatter(self, out, inp, async_op=False):
        if inp.numel() != out.numel() * self.world_size:
            raise ValueError("reduce_scatter: size mismatch")
        nb = out.numel() * out.element_size()
        ok = (inp.dtype == out.dtype and inp.dtype in (torch.float32, torch.bfloat16, torch.float16)
              and nb % 16 == 0 and self._pullable(out, inp, stage_bytes=nb * self.world_size))
        if not ok:
            return self.base.reduce_scatter(out, inp, async_op)
        if not out.is_contiguous():
            return self.base.reduce_scatter(out, inp, async_op)
        i = inp.contiguous()
        stage = self._next()
        ep, wgs = self.epoch, self._wgs(nb)
        return self._launch(lambda: torch.ops.xdot.ipc_reduce_scatter(i, out.view(-1), stage, self.sig_ptrs,
                                                                      self._status, self.rank, ep, self.ticks, wgs),
                            out, (i, out), async_op)

    # -- delegated ----------------------------------------------------------------------
    def all_reduce(self, t, op="sum", async_op=False):
        return self.base.all_reduce(t, op, async_op)

    def all_reduce_multi(self, ts, op="sum", async_op=False):
        return self.base.all_reduce_multi(ts, op, async_op)

    def broadcast(self, t, src=0, async_op=False):
        return self.base.broadcast(t, src, async_op)

    def all_gather_object(self, obj):
        return self.base.all_gather_object(obj)

    def barrier(self):
        self.base.barrier()

    def sendrecv(self, send, recv, dst, src, async_op=False):
        return self.base.sendrecv(send, recv, dst, src, async_op)

    def sendrecv_multi(self, pairs, async_op=False):
        return self.base.sendrecv_multi(pairs, async_op)

    def close(self) -> None:
        """Unmap the peers' pages and free this rank's (after a device sync and a barrier, so
        no peer is still reading them)."""
        if getattr(self, "_stage", None) is None:
            return
        torch.cuda.synchronize(self.device)
        self.base.barrier()
        ops = torch.ops.xdot
        for p in self._opened:
            ops.ipc_close(p)
        ops.ipc_free(self._stage)
        ops.ipc_free(self._sig)
        self._stage = self._sig = None
        self._opened = []
