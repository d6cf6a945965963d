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
