"""Stream ordering of every collective on the fused and ring paths (nothing else
exercises the async RCCL discipline on one GPU).  The same emulated 4-rank step runs twice:
with plain device-copy collectives, and with EmulatedComm's link model, where every collective
(all-gather, reduce-scatter, ring hop, all-reduce) runs on its own stream behind a spin of
bytes / (2 GB/s) — long enough that a consumer not ordered after its collective reads the
buffer before the data lands, or a producer overwrites a buffer still in flight.  Kernels are
deterministic, so both runs must agree bit for bit."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _step(comm, impl, chunks, dev):
    import xdot
    from xdot.parallel import GradSync

    torch.manual_seed(0)
    m = xdot.DistributedDotProductAttn(256, num_heads=4, impl=impl, chunk_plan=chunks, comm=comm).to(dev, torch.bfloat16)
    sync = GradSync(m, comm=comm, bucket_mb=0.05)
    g = torch.Generator(device="cpu").manual_seed(1)
    R, T = 300, 1200
    x = torch.randn(1, R, 256, generator=g).to(dev, torch.bfloat16).requires_grad_(True)
    mask = (torch.rand(1, R, T, generator=g) < 0.2).to(dev)
    mask[..., 0] = False
    out = m(x, x, x, mask)
    out.float().square().sum().backward()
    sync.wait()
    torch.cuda.synchronize()
    return [out.detach().clone(), x.grad.clone()] + [p.grad.clone() for p in m.parameters()]


@pytest.mark.parametrize("impl,chunks", [("flash", 1), ("flash", 2), ("ring", None)])
def test_link_model_matches_synchronous_collectives(gpu, impl, chunks):
    from xdot.utils.comm import EmulatedComm

    ref = _step(EmulatedComm(4, rank=1), impl, chunks, gpu)
    got = _step(EmulatedComm(4, rank=1, link_gbps=2.0, p2p_gbps=1.0), impl, chunks, gpu)
    for a, b in zip(ref, got):
        assert torch.equal(a, b)


def test_ring_peak_memory_independent_of_ring_length(gpu):
    """the ring path is the memory-lean one.  One rank (R = 2048 rows) of a 4- and of
    an 8-rank job (EmulatedComm): the flash path holds the whole gathered [q|v] side and its
    gradient partials, O(T); the ring holds two blocks, travelling fp32 accumulators and a
    running merge, O(R) — its peak must not grow with the ring length."""
    import xdot
    from xdot.utils.comm import EmulatedComm

    def peak(impl, n):
        comm = EmulatedComm(n, rank=0)
        torch.manual_seed(0)
        m = xdot.DistributedDotProductAttn(768, num_heads=8, impl=impl, comm=comm).to(gpu, torch.bfloat16)
        x = torch.randn(1, 2048, 768, device=gpu, dtype=torch.bfloat16)
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        base = torch.cuda.memory_allocated(gpu)
        torch.cuda.reset_peak_memory_stats(gpu)
        out = m(x, x, x, None)
        out.float().square().mean().backward()
        torch.cuda.synchronize()
        return torch.cuda.max_memory_allocated(gpu) - base

    f4, f8, r4, r8 = peak("flash", 4), peak("flash", 8), peak("ring", 4), peak("ring", 8)
    # 4 more ranks: 4 more (R, 2C) bf16 blocks of the gathered side and of its gradient partials
    grown = 2 * 4 * 2048 * 2 * 768 * 2
    assert f8 - f4 > 0.8 * grown, (f4, f8)
    assert abs(r8 - r4) < 0.1 * (f8 - f4), (r4, r8)
    assert r8 < f8, (r8, f8)


@pytest.mark.parametrize("link", [None, 2.0])
def test_fp32_weight_gradient_wire_matches_parameter_dtype_wire(gpu, monkeypatch, link):
    """GradSync(reduce_dtype=fp32) on a bf16 fused module (emulated 4-rank step, all-reduce = the
    local gradient): with the fp32 wire (XDOT_GRAD_WIRE32, default) the node hands over the weight
    gradients' fp32 sums and wait() rounds them into p.grad; without it the kernels round to bf16
    and GradSync converts to fp32 and back.  Same rounding of the same sums: p.grad bitwise equal.
    With FusedAdamW in the split step (the update reads the fp32 values and writes p.grad) the
    gradients stay bitwise equal and the parameters agree to bf16 rounding."""
    import xdot
    from xdot.parallel import GradSync
    from xdot.utils.comm import EmulatedComm
    from xdot.utils.env import FLAGS

    def run(wire, opt_step):
        monkeypatch.setattr(FLAGS, "grad_wire32", wire)
        comm = EmulatedComm(4, rank=1, link_gbps=link, p2p_gbps=link)
        torch.manual_seed(0)
        m = xdot.DistributedDotProductAttn(256, num_heads=4, comm=comm).to(gpu, torch.bfloat16)
        sync = GradSync(m, comm=comm, bucket_mb=0.05, reduce_dtype=torch.float32)
        opt = xdot.FusedAdamW(m.parameters(), lr=1e-3) if opt_step else None
        g = torch.Generator(device="cpu").manual_seed(3)
        x = torch.randn(1, 300, 256, generator=g).to(gpu, torch.bfloat16)
        m(x, x, x, None).float().square().sum().backward()
        if wire:
            assert sync._g32 and all(t.dtype == torch.float32 for t in sync._g32.values())
        else:
            assert not sync._g32
        stepped = sync.wait(optimizer=opt)
        assert stepped == opt_step
        torch.cuda.synchronize()
        return [p.grad.clone() for p in m.parameters()], [p.detach().clone() for p in m.parameters()]

    for opt_step in (False, True):
        g1, p1 = run(True, opt_step)
        g0, p0 = run(False, opt_step)
        for a, b in zip(g1, g0):
            assert a.dtype == torch.bfloat16 and torch.equal(a, b)
        for a, b in zip(p1, p0):
            torch.testing.assert_close(a.float(), b.float(), rtol=1e-2, atol=1e-4)
