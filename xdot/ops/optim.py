"""``FusedAdamW``: AdamW whose whole update is ONE HIP launch (``csrc/optim.hip``).

The reference trains the module with a stock optimizer; on MI355X torch's fused AdamW costs
≈50 µs per step for the module's 2.4M parameters (a few percent of an 8-GPU step).  This
optimizer keeps the moments in fp32 (also for bf16 parameters) and updates every parameter of
every group in one multi-tensor kernel per (group, dtype).  Semantics follow
``torch.optim.AdamW`` (decoupled weight decay, bias correction, ``amsgrad=False``); CPU
parameters and anything the kernel does not take fall back to ``torch.optim.AdamW``'s
functional update.

``capturable=True`` keeps the step count on the device (one fp32 scalar per parameter group
and dtype, advanced by a device op before each update, the bias corrections computed in the
kernel from it), so ``step()`` can be recorded in a HIP graph and replayed
(:class:`xdot.utils.graphs.GraphedStep`); every parameter of the group must then have a
gradient at every step.
"""
from __future__ import annotations

from typing import Iterable

import torch

from .. import _ext

__all__ = ["FusedAdamW"]


class FusedAdamW(torch.optim.Optimizer):
    def __init__(self, params: Iterable, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 1e-2, capturable: bool = False):
        if lr < 0 or eps < 0 or not (0 <= betas[0] < 1 and 0 <= betas[1] < 1) or weight_decay < 0:
            raise ValueError("invalid AdamW hyper-parameters")
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        self.capturable = capturable
        self._dev_step = {}  # (group index, dtype, device) -> fp32 device step count

    @torch.no_grad()
    def step(self, closure=None, params=None):
        """``params``: update only these parameters (each must then be updated once per step —
        :meth:`xdot.parallel.GradSync.wait` with ``optimizer=`` splits a step this way so the
        early buckets' update overlaps the last gradient all-reduce).  Not with ``capturable``."""
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        only = None
        if params is not None:
            if self.capturable:
                raise RuntimeError("FusedAdamW(capturable=True).step(params=...) is not supported")
            only = {id(p) for p in params}
        for gi, group in enumerate(self.param_groups):
            b1, b2 = group["betas"]
            buckets = {}
            for p in group["params"]:
                if p.grad is None or (only is not None and id(p) not in only):
                    continue
                st = self.state[p]
                if not st:
                    st["step"] = 0
                    st["exp_avg"] = torch.zeros_like(p, dtype=torch.float32, memory_format=torch.contiguous_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, dtype=torch.float32, memory_format=torch.contiguous_format)
                st["step"] += 1
                hip = (p.is_cuda and p.dtype in (torch.bfloat16, torch.float16, torch.float32) and p.is_contiguous()
                       and _ext.use_hip(p))
                if hip:
                    buckets.setdefault((p.dtype, p.device, 0 if self.capturable else st["step"]), []).append(p)
                elif self.capturable:
                    raise RuntimeError("FusedAdamW(capturable=True) needs contiguous bf16/fp16/fp32 GPU parameters")
                else:
                    self._torch_update(p, st, group, b1, b2)
            for (dt, dev, step), ps in buckets.items():
                step_t = None
                if self.capturable:
                    key = (gi, dt, dev)
                    step_t = self._dev_step.get(key)
                    if step_t is None:
                        step_t = self._dev_step[key] = torch.zeros((), dtype=torch.float32, device=dev)
                    step_t.add_(1.0)  # a device op: advances on every graph replay too
                    step = 1
                _ext.ops().adamw_step(ps, [p.grad.contiguous() for p in ps], [self.state[p]["exp_avg"] for p in ps],
                                      [self.state[p]["exp_avg_sq"] for p in ps], float(group["lr"]), float(b1),
                                      float(b2), float(group["eps"]), float(group["weight_decay"]), int(step), step_t)
        return loss

    @staticmethod
    def _torch_update(p, st, group, b1, b2):
        g = p.grad.float()
        m, v, t = st["exp_avg"], st["exp_avg_sq"], st["step"]
        m.mul_(b1).add_(g, alpha=1 - b1)
        v.mul_(b2).addcmul_(g, g, value=1 - b2)
        bc1, bc2 = 1 - b1 ** t, 1 - b2 ** t
        pf = p.float().mul_(1 - group["lr"] * group["weight_decay"])
        pf.addcdiv_(m, (v.sqrt() / bc2 ** 0.5).add_(group["eps"]), value=-group["lr"] / bc1)
        p.copy_(pf)
