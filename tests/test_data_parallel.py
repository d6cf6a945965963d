"""Replicated-parameter helpers: broadcast, bucketed Sum all-reduce, overlapped GradSync."""
import torch

from _dist import run_gloo


def _dp_body(rank, ws):
    from xdot.parallel import GradSync, allreduce_gradients, broadcast_parameters

    torch.manual_seed(rank)
    m = torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.Linear(16, 4))
    broadcast_parameters(m, bucket_mb=0.0001)  # tiny buckets: exercise bucketing
    ref = torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.Linear(16, 4))
    torch.manual_seed(0)
    ref0 = torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.Linear(16, 4))
    for p, q in zip(m.parameters(), ref0.parameters()):
        assert torch.equal(p, q), "broadcast from rank 0"
    # Sum all-reduce == gradient of the summed losses
    x = torch.full((3, 8), float(rank + 1))
    m(x).sum().backward()
    allreduce_gradients(m, bucket_mb=0.0001)
    ref.load_state_dict(m.state_dict())
    for r in range(ws):
        ref(torch.full((3, 8), float(r + 1))).sum().backward()
    for p, q in zip(m.parameters(), ref.parameters()):
        torch.testing.assert_close(p.grad, q.grad)
    # GradSync (hooks) gives the same result, also averaged
    for op in ("sum", "avg"):
        m.zero_grad()
        sync = GradSync(m, bucket_mb=0.0001, op=op)
        m(x).sum().backward()
        sync.wait()
        sync.remove()
        for p, q in zip(m.parameters(), ref.parameters()):
            torch.testing.assert_close(p.grad, q.grad / (ws if op == "avg" else 1))


def test_data_parallel_helpers_gloo():
    run_gloo(_dp_body, 2)


def test_single_rank_noops():
    from xdot.parallel import GradSync, allreduce_gradients, broadcast_parameters

    m = torch.nn.Linear(3, 3)
    w = m.weight.detach().clone()
    broadcast_parameters(m)
    m(torch.ones(1, 3)).sum().backward()
    g = m.weight.grad.clone()
    allreduce_gradients(m)
    sync = GradSync(m)
    sync.wait()
    assert torch.equal(m.weight, w) and torch.equal(m.weight.grad, g)
