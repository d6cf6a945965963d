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
