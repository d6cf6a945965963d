"""Replicated-parameter helpers for sequence-parallel training.

With time-axis sharding every rank holds a full replica of the (small) projection weights,
and each rank's parameter gradient is only the contribution of its own rows, so gradients
must be **summed** (not averaged) across ranks.  The reference leaves this to the user
(``tests/test_gradient.py:48`` ``hvd.broadcast_parameters``, ``:120``
``hvd.allreduce(param.grad, op=hvd.Sum)``); here it is a library feature:

* :func:`broadcast_parameters` — one flattened broadcast per dtype bucket;
* :func:`allreduce_gradients` — bucketed (flattened) Sum all-reduce, buckets sized for
  RCCL over xGMI (default 64 MiB: large enough to run the ring at link bandwidth);
* :class:`GradSync` — the same, but launched from per-parameter autograd hooks as soon as a
  bucket's gradients are ready, overlapping communication with the rest of backward.
"""
from __future__ import annotations

import contextlib
import functools
import inspect
from typing import Dict, Iterable, List, Optional

import torch
from torch import nn

from ..utils import comm as _comm

__all__ = ["broadcast_parameters", "allreduce_gradients", "GradSync"]


def _buckets(tensors: Iterable[torch.Tensor], bucket_bytes: int) -> List[List[torch.Tensor]]:
    by_key: Dict[tuple, List[List[torch.Tensor]]] = {}
    for t in tensors:
        key = (t.dtype, t.device)
        lst = by_key.setdefault(key, [[]])
        cur = lst[-1]
        if cur and sum(x.numel() * x.element_size() for x in cur) + t.numel() * t.element_size() > bucket_bytes:
            lst.append([])
            cur = lst[-1]
        cur.append(t)
    return [b for lst in by_key.values() for b in lst if b]


def _flat_apply(bucket: List[torch.Tensor], fn) -> None:
    flat = torch.cat([t.reshape(-1) for t in bucket])
    fn(flat)
    off = 0
    for t in bucket:
        n = t.numel()
        t.copy_(flat[off:off + n].view_as(t))
        off += n


@torch.no_grad()
def broadcast_parameters(module_or_tensors, src: int = 0, comm: Optional[_comm.Communicator] = None,
                         bucket_mb: float = 64.0) -> None:
    """Make every rank's parameters/buffers equal to rank ``src``'s."""
    comm = comm or _comm.get_comm()
    if comm.world_size == 1:
        return
    if isinstance(module_or_tensors, nn.Module):
        ts = list(module_or_tensors.state_dict().values())
    elif isinstance(module_or_tensors, dict):
        ts = list(module_or_tensors.values())
    else:
        ts = list(module_or_tensors)
    for b in _buckets(ts, int(bucket_mb * 2**20)):
        _flat_apply(b, lambda f: comm.broadcast(f, src=src))


@torch.no_grad()
def allreduce_gradients(module_or_params, op: str = "sum", comm: Optional[_comm.Communicator] = None,
                        bucket_mb: float = 64.0) -> None:
    """Sum (default) or average parameter gradients across ranks, bucketed."""
    comm = comm or _comm.get_comm()
    if comm.world_size == 1:
        return
    params = module_or_params.parameters() if isinstance(module_or_params, nn.Module) else module_or_params
    grads = [p.grad for p in params if p.grad is not None]
    ws = comm.world_size

    def red(f):
        comm.all_reduce(f, op="sum")
        if op == "avg":
            f.div_(ws)

    for b in _buckets(grads, int(bucket_mb * 2**20)):
        _flat_apply(b, red)


def _cast_into(srcs: List[torch.Tensor], dsts: List[torch.Tensor]) -> None:
    """``dst.copy_(src)`` for every pair (dtype conversion): ONE xdot launch for all the GPU pairs
    (csrc/optim.hip ``cast_multi``) instead of one elementwise kernel per tensor."""
    if not srcs:
        return
    from .. import _ext

    if dsts[0].is_cuda and _ext.use_hip(dsts[0]):
        _ext.ops().cast_multi([s.contiguous() for s in srcs], dsts)
        return
    for src, dst in zip(srcs, dsts):
        dst.copy_(src)


@functools.lru_cache(maxsize=None)
def _takes_params(opt_cls) -> bool:
    """Does ``opt_cls.step`` accept ``params=`` (a partial step, e.g. :class:`xdot.FusedAdamW`)?"""
    return "params" in inspect.signature(opt_cls.step).parameters


@functools.lru_cache(maxsize=None)
def _takes_grads(opt_cls) -> bool:
    """Does ``opt_cls.step`` also take ``grads=`` (fp32 gradients it writes into ``p.grad`` itself,
    :class:`xdot.FusedAdamW`)?"""
    return "grads" in inspect.signature(opt_cls.step).parameters



def _views(flat: torch.Tensor, params) -> List[torch.Tensor]:
    """Consecutive views of a flat bucket shaped like each parameter's gradient."""
    out, off = [], 0
    for p in params:
        n = p.numel()
        out.append(flat[off:off + n].view(p.shape))
        off += n
    return out

class GradSync:
    """Overlap gradient all-reduce with backward.

    Usage::

        sync = GradSync(model)          # registers hooks
        loss.backward()
        sync.wait()                     # all buckets reduced (stream-ordered)

    Contract (checked, never silently wrong):

    * one ``backward`` per ``wait()``.  A second backward before ``wait()`` would launch the
      all-reduces on partial gradients, so it raises; accumulate micro-batches under
      :meth:`no_sync` (hooks are muted there) and let the LAST backward run outside it;
    * every bucket must have been launched when ``wait()`` runs.  A parameter that requires a
      gradient but took no part in the backward leaves its bucket incomplete: ``unused="raise"``
      (default) raises naming it, ``unused="zero"`` reduces it as a zero gradient (every rank
      must then do the same, as with DDP's ``find_unused_parameters``);
    * ``reduce_dtype``: dtype of the all-reduce (e.g. ``torch.float32`` for bf16 gradients: one
      rounding at the end instead of one per ring step).  Default: the gradients' dtype.  A fused
      node asks :meth:`wire_dtype` and then hands over fp32 weight gradients of 16-bit parameters
      straight from its fp32 accumulators: they are reduced in place, and ``wait()`` writes
      ``p.grad`` once, rounded from the reduced fp32 sum (no conversion pass before the
      all-reduce, no rounding to 16 bits before the sum).
    """

    def __init__(self, module: nn.Module, comm: Optional[_comm.Communicator] = None,
                 bucket_mb: float = 16.0, op: str = "sum", reduce_dtype: Optional[torch.dtype] = None,
                 unused: str = "raise"):
        if op not in ("sum", "avg"):
            raise ValueError(f"op must be sum|avg, got {op!r}")
        if unused not in ("raise", "zero"):
            raise ValueError(f"unused must be raise|zero, got {unused!r}")
        self.comm = comm or _comm.get_comm()
        self.op = op
        self.reduce_dtype = reduce_dtype
        self.unused = unused
        params = [p for p in module.parameters() if p.requires_grad]
        self._names = {id(p): n for n, p in module.named_parameters()}
        # reverse registration order ~ gradient arrival order
        self.buckets = _buckets(list(reversed(params)), int(bucket_mb * 2**20))
        self._index = {id(p): i for i, b in enumerate(self.buckets) for p in b}
        self._seen = [set() for _ in self.buckets]
        self._launched = [False] * len(self.buckets)
        self._handles: List = []
        self._hooks = []
        self._muted = False
        self._rest_key = None
        self._held_key, self._held = None, set()
        self._batch = None  # buckets completed inside one deliver() call (launched together)
        self._rest: List[torch.Tensor] = []
        self._attached = []
        self._dlv = set()  # ids of parameters whose gradient was delivered this round
        self._g32 = {}     # id(p) -> fp32 gradient delivered for a 16-bit parameter (wire_dtype)
        self._uses = {}    # fused-module forwards since the last wait() (note_use / sole_use)
        if self.comm.world_size > 1:
            for p in params:
                self._hooks.append(p.register_post_accumulate_grad_hook(self._on_grad))
            # modules whose backward computes several parameter gradients in one autograd node
            # (xdot.models.fused.AttnBlockFn) hand each one over as soon as it exists (deliver),
            # so its all-reduce overlaps the rest of that node's backward
            import weakref

            for m in module.modules():
                if hasattr(m, "_xdot_grad_sync"):
                    m._xdot_grad_sync = weakref.ref(self)
                    self._attached.append(m)

    @contextlib.contextmanager
    def no_sync(self):
        """Accumulate gradients locally (no all-reduce) inside this context."""
        prev, self._muted = self._muted, True
        try:
            yield
        finally:
            self._muted = prev

    def note_use(self, key) -> None:
        """A fused node's forward (``key``: its module) ran with gradients enabled.  Forwards
        under :meth:`no_sync` are not counted: their backward runs muted and goes through
        AccumulateGrad, so only the forwards whose gradients are reduced decide :meth:`sole_use`."""
        if self._muted:
            return
        self._uses[key] = self._uses.get(key, 0) + 1

    def sole_use(self, key) -> bool:
        """Did ``key``'s module run exactly one forward since the last :meth:`wait`?  Only then
        may its node :meth:`deliver` gradients itself; a second use (the module called twice in
        one step) must leave the summing to autograd's AccumulateGrad."""
        return self._uses.get(key, 0) == 1

    def wire_dtype(self, p) -> torch.dtype:
        """dtype in which a fused node should hand ``p``'s gradient to :meth:`deliver`: fp32 for a
        16-bit parameter reduced here in fp32 this round (``reduce_dtype=torch.float32``, not under
        :meth:`no_sync`), else the parameter's own."""
        from ..utils.env import FLAGS

        if (FLAGS.grad_wire32 and self.reduce_dtype == torch.float32 and p.dtype in (torch.bfloat16, torch.float16)
                and not self._muted and self.comm.world_size > 1 and id(p) in self._index):
            return torch.float32
        return p.dtype

    @torch.no_grad()
    def deliver(self, pairs, stream=None) -> None:
        """Gradients computed early inside a multi-parameter backward node: accumulate each
        into ``p.grad`` (as autograd's AccumulateGrad would) and count it for its bucket, the
        bucket's all-reduce ordered after ``stream`` (where the gradients were computed).  The
        node then returns None for these parameters.  A gradient in :meth:`wire_dtype` fp32 for a
        16-bit parameter is held (and reduced) as is; :meth:`wait` writes ``p.grad`` from it."""
        cur = torch.cuda.current_stream() if stream is not None else None
        ctx = torch.cuda.stream(stream) if stream is not None else contextlib.nullcontext()
        with ctx:
            for p, g in pairs:
                if g is None:
                    continue
                if g.dtype != p.dtype:
                    if self.wire_dtype(p) == g.dtype:
                        if p.grad is not None:  # earlier micro-batches accumulated under no_sync()
                            g = g.add_(p.grad)
                        if cur is not None:
                            g.record_stream(cur)  # wait() writes p.grad from it on the current stream
                        self._g32[id(p)] = g
                        continue
                    g = g.to(p.dtype)
                if p.grad is None:
                    p.grad = g.detach()
                else:
                    p.grad.add_(g)
            if self._muted:  # no_sync(): accumulated only; NOT marked delivered, so the gradient of
                return       # a later unmuted backward through AccumulateGrad is still counted
            # buckets completed by this call are reduced together: ONE grouped collective for the
            # in-place ones (RCCL: one launch instead of one per bucket, each a small-message
            # latency on the step's tail)
            self._batch = []
            try:
                for p, g in pairs:
                    if g is not None and id(p) in self._index:  # (a parameter outside the buckets is
                        self._dlv.add(id(p))                   # accumulated, never reduced here)
                        self._on_grad(p, delivered=True)
                batch = self._batch
            finally:
                self._batch = None
            self._launch_many(batch)

    def _on_grad(self, p, delivered: bool = False):
        if self._muted:
            return
        if not delivered and id(p) in self._dlv:
            # autograd's AccumulateGrad still runs (with no gradient) for a parameter whose
            # gradient the node delivered itself, and its post-accumulate hook fires: ignore it
            return
        i = self._index[id(p)]
        if self._launched[i] or id(p) in self._seen[i]:
            raise RuntimeError(
                f"GradSync: gradient of {self._names.get(id(p), '<param>')} arrived again before wait(): "
                "run one backward per wait(), or accumulate earlier micro-batches under sync.no_sync()")
        self._seen[i].add(id(p))
        if len(self._seen[i]) == len(self.buckets[i]):
            if self._batch is not None:
                self._batch.append(i)
            else:
                self._launch(i)

    def _bucket_tensors(self, i):
        """(tensors to reduce, reduce dtype, in place?) of bucket i."""
        b = self.buckets[i]
        for p in b:
            if p.grad is None and id(p) not in self._g32:  # unused="zero": reduce a zero gradient
                p.grad = torch.zeros_like(p)
        ts = [self._g32[id(p)] if id(p) in self._g32 else p.grad for p in b]
        rdt = self.reduce_dtype or ts[0].dtype
        return ts, rdt, all(t.is_contiguous() and t.dtype == rdt for t in ts)

    def _launch_many(self, idx) -> None:
        """Launch buckets ``idx`` (completed together): the in-place ones as ONE grouped
        all-reduce (each bucket's entry shares its handle), the others one by one."""
        group = []
        for i in idx:
            ts, rdt, inplace = self._bucket_tensors(i)
            if inplace and (not group or group[0][2] == rdt):
                group.append((i, ts, rdt))
            else:
                self._launch(i)
        if len(group) < 2:
            for i, _, _ in group:
                self._launch(i)
            return
        nat = self.op == "avg" and self.comm.native_avg
        allt = [t for _, ts, _ in group for t in ts]
        h = self.comm.all_reduce_multi(allt, op="avg" if nat else "sum", async_op=True)
        for i, ts, _ in group:
            self._launched[i] = True
            back = [(t, p) for t, p in zip(ts, self.buckets[i]) if id(p) in self._g32]
            self._handles.append((i, ts, h, nat, back))

    def _launch(self, i):
        b = self.buckets[i]
        self._launched[i] = True
        ts, rdt, inplace = self._bucket_tensors(i)
        # "avg" in the collective itself where the backend has it (RCCL): no division pass
        nat = self.op == "avg" and self.comm.native_avg
        op = "avg" if nat else "sum"
        if inplace:
            # reduced in place (one grouped launch for a several-tensor bucket): no flatten pass;
            # the fp32 wire gradients are written into p.grad by wait()
            h = self.comm.all_reduce(ts[0], op=op, async_op=True) if len(b) == 1 else \
                self.comm.all_reduce_multi(ts, op=op, async_op=True)
            back = [(t, p) for t, p in zip(ts, b) if id(p) in self._g32]
            self._handles.append((i, ts, h, nat, back))
            return
        # converted straight into the flat buffer, every gradient of the bucket in one launch
        # (torch._foreach_copy_'s multi-tensor kernel ran ~14 us per 768 x 768 gradient on MI355X,
        # one elementwise copy per gradient ~5 us each: profiles/r6_fp32.md §4)
        flat = torch.empty(sum(p.numel() for p in b), dtype=rdt, device=ts[0].device)
        _cast_into(ts, _views(flat, b))
        h = self.comm.all_reduce(flat, op=op, async_op=True)
        self._handles.append((i, flat, h, nat, list(zip(_views(flat, b), b))))

    @torch.no_grad()
    def wait(self, optimizer=None) -> bool:
        """Order the current stream after every bucket's all-reduce.  With ``optimizer`` (one
        whose ``step`` takes ``params=``, e.g. :class:`xdot.FusedAdamW`) the update is split: the
        buckets reduced before the last one are stepped while the last all-reduce (the gradient
        that arrives last in backward) is still on the wire, then the last bucket together with
        every optimizer parameter outside the buckets.  Returns True when the optimizer has
        stepped (every parameter it holds, exactly once)."""
        ws = self.comm.world_size
        split = (optimizer is not None and ws > 1 and len(self._handles) > 1
                 and not getattr(optimizer, "capturable", False) and _takes_params(type(optimizer)))
        if ws > 1:
            missing = [i for i, done in enumerate(self._launched) if not done]
            if missing and self.unused == "raise":
                names = [self._names.get(id(p), "<param>") for i in missing for p in self.buckets[i]
                         if id(p) not in self._seen[i]]
                self._reset()
                raise RuntimeError(f"GradSync.wait(): no gradient arrived for {names} (unused parameter? "
                                   "freeze it, or pass unused='zero')")
            for i in missing:  # bucket index order: the same on every rank
                self._launch(i)
        last = len(self._handles) - 1
        back = []  # (reduced tensor, parameter) pairs whose p.grad is written in one launch
        for k, (i, flat, h, nat, bk) in enumerate(self._handles):
            if split and k == last:  # everything reduced so far steps under the last all-reduce
                self._step_with(optimizer, [p for j, *_ in self._handles[:last] for p in self.buckets[j]], back)
                back = []
            h.wait()
            if self.op == "avg" and not nat:
                if isinstance(flat, list):  # reduced in place
                    torch._foreach_div_(flat, ws)
                else:
                    flat.div_(ws)
            back.extend(bk)
        if split:
            rest = self._outside_params(optimizer)
            self._step_with(optimizer, list(self.buckets[self._handles[last][0]]) + rest, back)
        else:
            self._write_back(back)
        self._reset()
        return split

    def _step_with(self, optimizer, params, back) -> None:
        """``optimizer.step(params=params)`` after writing the reduced values of ``back`` into
        ``p.grad`` -- by the optimizer itself where it takes fp32 ``grads=`` (FusedAdamW: the write-
        back folded into its update launch), else in one :meth:`_write_back` launch."""
        over = {}
        if back and _takes_grads(type(optimizer)):
            held = self._held_ids(optimizer)
            over = {id(p): t for t, p in back if id(p) in held and t.dtype == torch.float32
                    and p.dtype in (torch.bfloat16, torch.float16)}
        self._write_back([(t, p) for t, p in back if id(p) not in over])
        if over:
            optimizer.step(params=params, grads=[over.get(id(p)) for p in params])
        else:
            optimizer.step(params=params)

    @staticmethod
    def _write_back(pairs) -> None:
        """p.grad <- the reduced values (rounded to p's dtype), every pair in one launch."""
        for _, p in pairs:
            if p.grad is None:
                p.grad = torch.empty_like(p)
        ok = [(t, p) for t, p in pairs if p.grad.is_contiguous()]
        _cast_into([t for t, _ in ok], [p.grad for _, p in ok])
        for t, p in pairs:
            if not p.grad.is_contiguous():  # (a .grad the user set as a strided view)
                p.grad.copy_(t)

    def _held_ids(self, optimizer) -> set:
        """ids of the parameters ``optimizer`` holds (cached per optimizer and parameter count)."""
        key = (id(optimizer), sum(len(g["params"]) for g in optimizer.param_groups))
        if self._held_key != key:
            self._held = {id(p) for g in optimizer.param_groups for p in g["params"]}
            self._held_key = key
        return self._held

    def _outside_params(self, optimizer) -> List[torch.Tensor]:
        """Parameters the optimizer holds that are not in this GradSync's buckets (a second
        module, an extra param group, a parameter outside ``module.parameters()``): a split
        step must update them too, else they would silently never train.  Cached per
        (optimizer, parameter count)."""
        key = (id(optimizer), sum(len(g["params"]) for g in optimizer.param_groups))
        if self._rest_key != key:
            mine = {id(p) for b in self.buckets for p in b}
            self._rest = [p for g in optimizer.param_groups for p in g["params"]
                          if id(p) not in mine and p.requires_grad]
            self._rest_key = key
        return self._rest

    def _reset(self):
        self._handles.clear()
        self._dlv = set()
        self._g32 = {}
        self._uses = {}
        self._seen = [set() for _ in self.buckets]
        self._launched = [False] * len(self.buckets)

    def remove(self):
        for h in self._hooks:
            h.remove()
        self._hooks.clear()
        for m in self._attached:
            m._xdot_grad_sync = None
        self._attached.clear()
