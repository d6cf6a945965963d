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


def test_step_hooks_and_profiler_range_still_work():
    """FusedAdamW.step skips torch's profiling wrapper only while nothing observes it: step
    hooks (per optimizer and global) still run, and a profiler still sees the step range."""
    from torch.optim.optimizer import register_optimizer_step_pre_hook

    p = torch.zeros(3, requires_grad=True)
    opt = FusedAdamW([p], lr=1e-2)
    assert getattr(FusedAdamW.step, "hooked", False)
    seen = []
    h1 = opt.register_step_pre_hook(lambda o, a, k: seen.append("pre"))
    h2 = opt.register_step_post_hook(lambda o, a, k: seen.append("post"))
    h3 = register_optimizer_step_pre_hook(lambda o, a, k: seen.append("global"))
    p.grad = torch.ones(3)
    opt.step()
    assert seen == ["global", "pre", "post"]
    h1.remove(); h2.remove(); h3.remove()
    seen.clear()
    p.grad = torch.ones(3)
    opt.step()
    assert seen == [] and torch.is_grad_enabled()
    with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU]) as prof:
        p.grad = torch.ones(3)
        opt.step()
    assert any("Optimizer.step#FusedAdamW.step" in e.key for e in prof.key_averages())
    # the step ran under no_grad either way
    assert not p.grad.requires_grad and torch.is_grad_enabled()


def test_step_closure_and_params_subset():
    g = torch.Generator().manual_seed(1)
    a, b = torch.randn(4, generator=g).requires_grad_(True), torch.randn(4, generator=g).requires_grad_(True)
    a0, b0 = a.detach().clone(), b.detach().clone()
    opt = FusedAdamW([a, b], lr=1e-2)

    def closure():
        opt.zero_grad()
        loss = (a * a).sum() + (b * b).sum()
        loss.backward()
        return loss

    loss = opt.step(closure)
    assert torch.is_tensor(loss) and not torch.equal(a.detach(), a0) and not torch.equal(b.detach(), b0)
    a1, b1 = a.detach().clone(), b.detach().clone()
    a.grad, b.grad = torch.ones(4), torch.ones(4)
    opt.step(params=[a])
    assert not torch.equal(a.detach(), a1) and torch.equal(b.detach(), b1)
