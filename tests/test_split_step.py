"""GradSync.wait(optimizer=...) splits the optimizer step around the last all-reduce: the result
must equal one full step after every all-reduce (CPU, 2 gloo ranks)."""
import torch

from _dist import run_gloo


def _case(rank, ws):
    import xdot
    from xdot.parallel import GradSync

    def run(split):
        torch.manual_seed(0)
        m = xdot.DistributedDotProductAttn(64, num_heads=2, impl="materialized")
        opt = xdot.FusedAdamW(m.parameters(), lr=1e-2)
        sync = GradSync(m, bucket_mb=0.001)  # one bucket per parameter
        g = torch.Generator().manual_seed(10 + rank)
        for _ in range(3):
            x = torch.randn(1, 16, 64, generator=g)
            opt.zero_grad(set_to_none=True)
            m(x, x, x, None).square().mean().backward()
            stepped = sync.wait(optimizer=opt if split else None)
            assert stepped == split
            if not stepped:
                opt.step()
        return [p.detach().clone() for p in m.parameters()]

    for a, b in zip(run(False), run(True)):
        assert torch.equal(a, b)


def test_split_step_matches_full_step():
    run_gloo(_case, 2)


def _case_extra(rank, ws):
    """The optimizer holds a parameter outside the synced module (and a second param group):
    the split step still updates it, exactly as a full step would."""
    import xdot
    from xdot.parallel import GradSync

    def run(split):
        torch.manual_seed(0)
        m = xdot.DistributedDotProductAttn(64, num_heads=2, impl="materialized")
        extra = torch.nn.Parameter(torch.randn(5))
        run.init = extra.detach().clone()
        opt = xdot.FusedAdamW([{"params": list(m.parameters())}, {"params": [extra], "lr": 5e-2}], lr=1e-2)
        sync = GradSync(m, bucket_mb=0.001)
        g = torch.Generator().manual_seed(10 + rank)
        for _ in range(3):
            x = torch.randn(1, 16, 64, generator=g)
            opt.zero_grad(set_to_none=True)
            (m(x, x, x, None).square().mean() + extra.square().sum()).backward()
            stepped = sync.wait(optimizer=opt if split else None)
            assert stepped == split
            if not stepped:
                opt.step()
        return [p.detach().clone() for p in m.parameters()] + [extra.detach().clone()]

    a, b = run(False), run(True)
    assert not torch.equal(b[-1], run.init), "extra parameter never moved"
    for x, y in zip(a, b):
        assert torch.equal(x, y)


def test_split_step_updates_params_outside_the_buckets():
    run_gloo(_case_extra, 2)
