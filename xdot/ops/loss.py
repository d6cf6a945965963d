"""Fused mean-squared-error loss (the training loss of the reference's ``example.py`` /
``benchmark.py`` runs, ``torch.nn.MSELoss()``).

GPU tensors: one pass of ``csrc/reduce.hip::mse_fwd_kernel`` reads the prediction and target
once, writes the gradient ``2 (y - t) / n`` in the input dtype and per-workgroup fp32 partial
sums, and ``mse_final_kernel`` sums those partials in a fixed order (deterministic) into the
mean.  The backward only scales the saved gradient by the incoming one.  torch's chain for the
same loss is five to seven kernels per step (difference, square, mean reduction, a second pass
over prediction and target in the backward, fills); at the N=8 rank shape it cost ≈46 µs of a
≈1.4 ms step.  CPU tensors and layouts the kernel does not take use ``F.mse_loss``.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn.functional as F

from .. import _ext

__all__ = ["mse_loss", "MSELoss", "unit_grad"]

_DT = (torch.bfloat16, torch.float16, torch.float32)


def _hip_ok(y: torch.Tensor, t: torch.Tensor) -> bool:
    return (_ext.use_hip(y, t) and y.dtype in _DT and t.dtype == y.dtype and y.shape == t.shape and
            y.is_contiguous() and t.is_contiguous() and y.numel() > 0 and
            y.numel() % (16 // y.element_size()) == 0 and
            y.data_ptr() % 16 == 0 and t.data_ptr() % 16 == 0)


class _MSE(torch.autograd.Function):
    @staticmethod
    @_ext.pinned
    def forward(ctx, y, t):
        loss, dy = _ext.ops().mse_fwd(y, t)
        ctx.save_for_backward(dy)
        return loss

    @staticmethod
    @_ext.pinned
    def backward(ctx, g):
        (dy,) = ctx.saved_tensors
        # an exact-1 seed (unit_grad) leaves the saved gradient as it is: no scaling pass
        gy = dy if getattr(g, "_xdot_unit", False) else dy * g.to(dy.dtype)
        gt = -gy if ctx.needs_input_grad[1] else None
        return (gy if ctx.needs_input_grad[0] else None), gt


_UNIT = {}


def unit_grad(loss: torch.Tensor) -> torch.Tensor:
    """A cached exact-1 seed for ``loss.backward(unit_grad(loss))``: the same gradient as
    ``loss.backward()`` without autograd's per-call fill of a ones tensor, and the fused loss
    hands its saved gradient on without the scaling pass (two small kernels per step).  The
    returned tensor is shared: do not modify it."""
    key = (loss.device, loss.dtype, tuple(loss.shape))
    t = _UNIT.get(key)
    if t is None:
        t = _UNIT[key] = torch.ones(loss.shape, dtype=loss.dtype, device=loss.device)
        t._xdot_unit = True
    return t


def backward(loss: torch.Tensor, grad: Optional[torch.Tensor] = None, inline: Optional[bool] = None) -> None:
    """``loss.backward(grad)``, by default on the calling thread (``XDOT_INLINE_BACKWARD=1``).

    For GPU tensors PyTorch's autograd engine runs the backward on a per-device worker thread
    while the caller waits; the hand-off (and the GIL ping-pong for every Python backward
    function) costs ~0.2 ms of host time per step at the N=8 rank shape, where the GPU step is
    ~1.35 ms (profiles/r4_s2.md).  ``torch.autograd.set_multithreading_enabled(False)`` runs the
    same graph, in the same order and on the same streams, on this thread."""
    from ..utils.env import FLAGS

    if inline is None:
        inline = FLAGS.inline_backward
    if not inline:
        loss.backward(grad)
        return
    with torch.autograd.set_multithreading_enabled(False):
        loss.backward(grad)


def mse_loss(input: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
    """``mean((input - target) ** 2)`` (``reduction='mean'``), fused on the GPU."""
    if _hip_ok(input, target):
        return _MSE.apply(input, target)
    return F.mse_loss(input, target)


class MSELoss(torch.nn.Module):
    """Drop-in for ``torch.nn.MSELoss()`` (mean reduction)."""

    def forward(self, input: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
        return mse_loss(input, target)
