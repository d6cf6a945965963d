"""HIP-graph capture of a whole training step (forward + backward + optimizer), replayed with
one launch.

On MI355X a step of the module enqueues ≈27 kernels plus collectives from Python; at small
per-rank work (short sequences, many ranks) the host's ≈0.76 ms of enqueue time per step
(`bench.py`'s ``host_enqueue_ms_per_step``) exceeds the GPU time and the step becomes
launch-bound.  :class:`GraphedStep` records the step once into a ``torch.cuda.CUDAGraph`` (HIP
graph under ROCm) — side streams (the backward's priority stream, collective link streams)
fork from and join the capture stream, allocations come from the graph's private pool — and
replays it: no Python, no per-kernel launch cost.

Requirements (checked by use, as for any graph capture): static input tensors (copy new data
into them), static shapes, a capturable optimizer (``FusedAdamW(capturable=True)``: the step
count lives on the device), no host reads of device values inside the step, and a
communicator whose collectives are capturable (the single-GPU / emulated communicators, and
RCCL through ``TorchDistComm``: all-reduce / all-gather / reduce-scatter captured and replayed
in ``scripts/rccl_graph_check.py``, ``tests/test_rccl_gpu.py``; ``bench.py --graph`` under
torchrun with the nccl backend: 8.19 ms, 0.018 ms host per step, ``profiles/r4_s2.md`` §22 —
world size 1 on the one-GPU box; the multi-GPU capture is the same calls).  Gradients are allocated inside the capture
(``zero_grad(set_to_none=True)`` happens before it), so after a replay ``p.grad`` holds that
step's gradient.
"""
from __future__ import annotations

from typing import Callable, Optional

import torch

__all__ = ["GraphedStep"]


class GraphedStep:
    """``GraphedStep(step_fn, zero_grad=opt.zero_grad, optimizer=opt)``: ``step_fn()`` runs one training step and
    returns the loss tensor.  The first call runs ``warmup`` eager steps on a side stream,
    captures one step and replays it (``warmup + 1`` training steps); every later call replays
    it once.  Returns the (static) loss tensor of the step just run."""

    def __init__(self, step_fn: Callable[[], torch.Tensor], zero_grad: Optional[Callable[..., None]] = None,
                 warmup: int = 3, device: Optional[torch.device] = None, optimizer=None):
        if warmup < 1:
            # the optimizer's lazy state (moments, device step counts) must exist before the
            # capture, else every replay would re-create it and train as step 1 forever
            raise ValueError("GraphedStep needs warmup >= 1 (optimizer state is created by the eager steps)")
        self.step_fn = step_fn
        self.optimizer = optimizer
        self.zero_grad = zero_grad
        self.warmup = warmup
        self.device = device
        self.graph: Optional[torch.cuda.CUDAGraph] = None
        self.loss: Optional[torch.Tensor] = None

    def _zero(self):
        if self.zero_grad is not None:
            self.zero_grad(set_to_none=True)

    def capture(self) -> None:
        dev = self.device or torch.device("cuda", torch.cuda.current_device())
        side = torch.cuda.Stream(device=dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):  # eager warmup (allocator / kernel selection) off the default stream
            for _ in range(self.warmup):
                self._zero()
                self.step_fn()
        torch.cuda.current_stream(dev).wait_stream(side)
        if self.optimizer is not None and getattr(self.optimizer, "capturable", None) is False:
            raise ValueError("GraphedStep: the optimizer must be capturable (e.g. FusedAdamW(capturable=True))")
        self._zero()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, capture_error_mode="relaxed"):
            self.loss = self.step_fn()
        self.graph = g

    def __call__(self) -> torch.Tensor:
        if self.graph is None:
            self.capture()  # the warmup steps + the captured step are real training steps
        if self.optimizer is not None and hasattr(self.optimizer, "sync_lr"):
            self.optimizer.sync_lr()  # lr schedulers: the captured update reads lr from the device
        self.graph.replay()
        return self.loss
