"""HIP-graph captured training step (xdot.utils.graphs.GraphedStep + FusedAdamW(capturable=True))
vs the same steps run eagerly: losses and parameters agree."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _train(gpu, graphed, steps=5, warmup=2):
    import xdot
    from xdot.utils.graphs import GraphedStep

    torch.manual_seed(0)
    m = xdot.DistributedDotProductAttn(256, num_heads=4, impl="flash").to(gpu, torch.bfloat16)
    opt = xdot.FusedAdamW(m.parameters(), lr=1e-3, capturable=graphed)
    crit = xdot.MSELoss()
    g = torch.Generator(device=gpu).manual_seed(1)
    x = torch.rand(1, 512, 256, device=gpu, dtype=torch.bfloat16, generator=g)
    y = torch.rand(1, 512, 256, device=gpu, dtype=torch.bfloat16, generator=g)
    mask = torch.rand(1, 512, 512, device=gpu, generator=g) < 0.2
    mask[..., 0] = False

    def body():
        loss = crit(m(x, x, x, mask), y)
        loss.backward()
        opt.step()
        return loss

    losses = []
    if graphed:
        st = GraphedStep(body, zero_grad=opt.zero_grad, warmup=warmup)
        losses.append(st().float().item())          # warmup + 1 steps
        for _ in range(steps - warmup - 1):
            losses.append(st().float().item())
    else:
        for i in range(steps):
            opt.zero_grad(set_to_none=True)
            l = body().float().item()
            if i >= warmup:
                losses.append(l)
    torch.cuda.synchronize()
    return losses, [p.detach().float().clone() for p in m.parameters()]


def test_graphed_step_matches_eager(gpu):
    le, pe = _train(gpu, False)
    lg, pg = _train(gpu, True)
    assert len(le) == len(lg) == 3
    for a, b in zip(le, lg):
        assert abs(a - b) <= 2e-2 * abs(a) + 1e-6, (le, lg)
    for a, b in zip(pe, pg):
        assert ((a - b).norm() / a.norm()).item() < 1e-2
    # replays keep training: the parameters moved between steps
    _, p1 = _train(gpu, True, steps=4)
    assert any((a - b).abs().max().item() > 0 for a, b in zip(p1, pg))


def _adam_run(gpu, steps, resume_at=None, capturable=True):
    import xdot

    torch.manual_seed(0)
    w = torch.nn.Parameter(torch.randn(1000, device=gpu))
    opt = xdot.FusedAdamW([w], lr=1e-2, capturable=capturable)
    g = torch.Generator(device=gpu).manual_seed(3)
    grads = [torch.randn(1000, device=gpu, generator=g) for _ in range(steps)]
    for i in range(steps):
        if resume_at is not None and i == resume_at:
            sd = opt.state_dict()
            opt = xdot.FusedAdamW([w], lr=1e-2, capturable=capturable)
            opt.load_state_dict(sd)
        w.grad = grads[i].clone()
        opt.step()
    torch.cuda.synchronize()
    return w.detach().clone(), opt


def test_capturable_adamw_state_round_trips(gpu):
    """state['step'] of a capturable FusedAdamW lives on the device and survives
    state_dict/load_state_dict: a resumed run equals a continuous one (no bias-correction
    restart), and equals the non-capturable optimizer."""
    a, opt = _adam_run(gpu, 4)
    b, _ = _adam_run(gpu, 4, resume_at=2)
    c, _ = _adam_run(gpu, 4, capturable=False)
    assert torch.equal(a, b)
    torch.testing.assert_close(a, c, rtol=1e-5, atol=1e-6)
    st = opt.state_dict()["state"][0]["step"]
    assert torch.is_tensor(st) and float(st) == 4.0


def test_graphed_step_follows_lr_changes(gpu):
    """The captured update reads lr from the device: changing group['lr'] between replays
    (an LR scheduler) takes effect; lr = 0 freezes the parameters."""
    import xdot
    from xdot.utils.graphs import GraphedStep

    torch.manual_seed(0)
    w = torch.nn.Parameter(torch.randn(256, device=gpu))
    opt = xdot.FusedAdamW([w], lr=1e-2, weight_decay=0.0, capturable=True)
    x = torch.randn(256, device=gpu)

    def body():
        loss = (w * x).sum()
        loss.backward()
        opt.step()
        return loss

    st = GraphedStep(body, zero_grad=opt.zero_grad, warmup=1, optimizer=opt)
    st()
    w1 = w.detach().clone()
    opt.param_groups[0]["lr"] = 0.0
    st()
    torch.cuda.synchronize()
    assert torch.equal(w.detach(), w1)
    opt.param_groups[0]["lr"] = 1e-2
    st()
    torch.cuda.synchronize()
    assert not torch.equal(w.detach(), w1)
