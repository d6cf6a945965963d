"""FusedAdamW == torch.optim.AdamW (CPU path here; the HIP kernel in test_kernels_gpu.py)."""
import torch

from xdot.ops.optim import FusedAdamW


def _run(opt_cls, params, grads, steps, **kw):
    ps = [p.clone().requires_grad_(True) for p in params]
    opt = opt_cls(ps, **kw)
    for s in range(steps):
        for p, g in zip(ps, grads):
            p.grad = g * (s + 1)
        opt.step()
    return ps


def test_fused_adamw_matches_torch_cpu():
    g = torch.Generator().manual_seed(0)
    params = [torch.randn(7, 5, generator=g), torch.randn(13, generator=g)]
    grads = [torch.randn_like(p) for p in params]
    kw = dict(lr=1e-2, betas=(0.9, 0.99), eps=1e-6, weight_decay=0.1)
    a = _run(FusedAdamW, params, grads, 4, **kw)
    b = _run(torch.optim.AdamW, params, grads, 4, **kw)
    for x, y in zip(a, b):
        torch.testing.assert_close(x, y, rtol=1e-5, atol=1e-6)


def test_graphed_step_rejects_zero_warmup():
    import pytest

    from xdot.utils.graphs import GraphedStep

    with pytest.raises(ValueError):
        GraphedStep(lambda: None, warmup=0)
