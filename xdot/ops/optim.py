"""``FusedAdamW``: AdamW whose whole update is ONE HIP launch (``csrc/optim.hip``).

The reference trains the module with a stock optimizer; on MI355X torch's fused AdamW costs
≈50 µs per step for the module's 2.4M parameters (a few percent of an 8-GPU step).  This
optimizer keeps the moments in fp32 (also for bf16 parameters) and updates every parameter of
every group in one multi-tensor kernel per (group, dtype).  Semantics follow
``torch.optim.AdamW`` (decoupled weight decay, bias correction, ``amsgrad=False``); CPU
parameters and anything the kernel does not take fall back to ``torch.optim.AdamW``'s
functional update.

``capturable=True`` keeps the optimizer state the update reads on the device, as
``torch.optim.AdamW(capturable=True)`` does: every parameter's ``state["step"]`` is a 0-d fp32
device tensor (advanced by one multi-tensor device op before each update, the bias corrections
computed in the kernel from it; it round-trips through ``state_dict``/``load_state_dict`` and a
resumed run continues its bias correction), and each param group's learning rate lives in a
one-element device tensor that :meth:`FusedAdamW.sync_lr` refreshes from ``group["lr"]``.  So
``step()`` can be recorded in a HIP graph and replayed (:class:`xdot.utils.graphs.GraphedStep`
calls ``sync_lr`` before every replay, so LR schedulers keep working); every parameter of the
group must then have a gradient at every step.  ``weight_decay``/``betas``/``eps`` are baked in
at capture time.
"""
from __future__ import annotations

from typing import Iterable

import torch

from .. import _ext

from torch.optim import optimizer as _optim_mod

__all__ = ["FusedAdamW"]


class FusedAdamW(torch.optim.Optimizer):
    def __init__(self, params: Iterable, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 1e-2, capturable: bool = False):
        if lr < 0 or eps < 0 or not (0 <= betas[0] < 1 and 0 <= betas[1] < 1) or weight_decay < 0:
            raise ValueError("invalid AdamW hyper-parameters")
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        self.capturable = capturable
        self._lr_dev = {}  # (group index, device) -> one-element fp32 device tensor (capturable)

    def zero_grad(self, set_to_none: bool = True) -> None:
        """``set_to_none`` (the default): drop every gradient with a plain loop (the base class
        wraps the same work in a profiler range and per-device grouping: ~15 µs of host per
        step at the module's 8 parameters)."""
        if not set_to_none:
            return super().zero_grad(set_to_none=False)
        for group in self.param_groups:
            for p in group["params"]:
                p.grad = None

    def step(self, closure=None, params=None, grads=None):
        """``params``: update only these parameters (each must then be updated once per step —
        :meth:`xdot.parallel.GradSync.wait` with ``optimizer=`` splits a step this way so the
        early buckets' update overlaps the last gradient all-reduce).  Not with ``capturable``.
        ``grads`` (with ``params``, aligned, entries may be None): fp32 gradients to use instead of
        ``p.grad`` for 16-bit parameters (GradSync's reduced fp32 sums); the kernel also writes each
        into ``p.grad``, rounded to the parameter dtype (GradSync's write-back pass folded into the
        update).

        torch wraps every optimizer's ``step`` in a profiler range plus the step-hook loops
        (``Optimizer.profile_hook_step``): ~35 µs of host per call, twice per training step when
        the step is split around the last all-reduce.  This class opts out of that wrapper
        (``step.hooked`` below) and takes torch's wrapped path only when something would observe
        it: a registered step hook (per optimizer or global) or an active autograd profiler."""
        if (self._optimizer_step_pre_hooks or self._optimizer_step_post_hooks or _optim_mod._global_optimizer_pre_hooks
                or _optim_mod._global_optimizer_post_hooks or torch.autograd._profiler_enabled()):
            return _hooked_step(self, closure, params, grads)
        prev = torch.is_grad_enabled()
        torch._C._set_grad_enabled(False)
        try:
            return self._step_impl(closure, params, grads)
        finally:
            torch._C._set_grad_enabled(prev)

    step.hooked = True  # torch.optim.Optimizer._patch_step_function: leave this step unwrapped

    def _step_impl(self, closure=None, params=None, grads=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        only = None
        over = {}  # id(p) -> fp32 gradient replacing p.grad (written into p.grad by the update)
        if params is not None:
            if self.capturable:
                raise RuntimeError("FusedAdamW(capturable=True).step(params=...) is not supported")
            params = list(params)
            only = {id(p) for p in params}
            if grads is not None:
                over = {id(p): g for p, g in zip(params, grads) if g is not None}
        elif grads is not None:
            raise ValueError("FusedAdamW.step(grads=...) needs params=")
        for gi, group in enumerate(self.param_groups):
            b1, b2 = group["betas"]
            buckets = {}
            for p in group["params"]:
                if only is not None and id(p) not in only:
                    continue
                g32 = over.get(id(p))
                if g32 is not None:
                    if p.grad is None:
                        p.grad = torch.empty_like(p)
                    if not (g32.dtype == torch.float32 and p.dtype in (torch.bfloat16, torch.float16)
                            and g32.is_contiguous() and p.grad.is_contiguous() and g32.shape == p.shape):
                        p.grad.copy_(g32)  # (the kernel takes fp32 gradients of 16-bit parameters only)
                        g32 = None
                if p.grad is None:
                    continue
                st = self.state[p]
                if not st:
                    st["step"] = torch.zeros((), dtype=torch.float32, device=p.device) if self.capturable else 0
                    st["exp_avg"] = torch.zeros_like(p, dtype=torch.float32, memory_format=torch.contiguous_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, dtype=torch.float32, memory_format=torch.contiguous_format)
                hip = (p.is_cuda and p.dtype in (torch.bfloat16, torch.float16, torch.float32) and p.is_contiguous()
                       and _ext.use_hip(p))
                if self.capturable:
                    if not hip:
                        raise RuntimeError("FusedAdamW(capturable=True) needs contiguous bf16/fp16/fp32 GPU parameters")
                    st["step"] = self._dev_step_of(st["step"], p.device)
                    buckets.setdefault((p.dtype, p.device, 0, False), []).append(p)
                    continue
                if torch.is_tensor(st["step"]):  # a state loaded from a capturable optimizer
                    st["step"] = int(st["step"].item())
                st["step"] += 1
                if hip:
                    buckets.setdefault((p.dtype, p.device, st["step"], g32 is not None), []).append(p)
                else:
                    if g32 is not None:
                        p.grad.copy_(g32)
                    self._torch_update(p, st, group, b1, b2)
            for (dt, dev, step, ov), ps in buckets.items():
                steps, lr_t = [], None
                if self.capturable:
                    steps = [self.state[p]["step"] for p in ps]
                    torch._foreach_add_(steps, 1.0)  # device ops: advance on every graph replay too
                    lr_t = self._lr_tensor(gi, group, dev)
                    step = 1
                gs = [over[id(p)] for p in ps] if ov else [p.grad.contiguous() for p in ps]
                _ext.ops().adamw_step(ps, gs, [self.state[p]["exp_avg"] for p in ps],
                                      [self.state[p]["exp_avg_sq"] for p in ps], float(group["lr"]), float(b1),
                                      float(b2), float(group["eps"]), float(group["weight_decay"]), int(step),
                                      steps, lr_t, [p.grad for p in ps] if ov else [])
        return loss

    @staticmethod
    def _dev_step_of(step, device) -> torch.Tensor:
        """The parameter's step count as a 0-d fp32 device tensor (seeded from a loaded int or
        tensor state, so a resumed run continues its bias correction)."""
        if torch.is_tensor(step):
            if step.device == device and step.dtype == torch.float32 and step.dim() == 0:
                return step
            return step.detach().reshape(()).to(device=device, dtype=torch.float32)
        return torch.full((), float(step), dtype=torch.float32, device=device)

    def _lr_tensor(self, gi, group, dev) -> torch.Tensor:
        t = self._lr_dev.get((gi, dev))
        if t is None:
            t = self._lr_dev[(gi, dev)] = torch.full((1,), float(group["lr"]), dtype=torch.float32, device=dev)
        elif not torch.cuda.is_current_stream_capturing():
            t.fill_(float(group["lr"]))  # eager step: follow the group's current lr
        return t

    def sync_lr(self) -> None:
        """Copy every param group's current ``lr`` into its device tensor (capturable mode; call
        before replaying a captured step so schedulers take effect — GraphedStep does)."""
        for (gi, _dev), t in self._lr_dev.items():
            t.fill_(float(self.param_groups[gi]["lr"]))

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        if self.capturable:  # re-home loaded step counts on the parameters' devices now
            for group in self.param_groups:
                for p in group["params"]:
                    st = self.state.get(p)
                    if st and "step" in st:
                        st["step"] = self._dev_step_of(st["step"], p.device)

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


@torch.no_grad()
def _unwrapped_step(self, closure=None, params=None, grads=None):
    return self._step_impl(closure, params, grads)


# torch's own wrapper (profiler range + pre/post step hooks) around the same update, for the
# calls that something observes
_hooked_step = torch.optim.Optimizer.profile_hook_step(_unwrapped_step)

