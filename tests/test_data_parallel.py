"""Replicated-parameter helpers: broadcast, bucketed Sum all-reduce, overlapped GradSync."""
import pytest
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


def _gradsync_contract_body(rank, ws):
    import pytest
    from xdot.parallel import GradSync

    torch.manual_seed(0)
    m = torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.Linear(16, 4))
    x = torch.full((3, 8), float(rank + 1))

    def summed_grads(xs):
        ref = torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.Linear(16, 4))
        ref.load_state_dict(m.state_dict())
        for xx in xs:
            ref(xx).sum().backward()
        return [p.grad for p in ref.parameters()]

    all_x = [torch.full((3, 8), float(r + 1)) for r in range(ws)]
    # frozen parameter: excluded from the buckets, no error, no gradient
    m[0].bias.requires_grad_(False)
    sync = GradSync(m, bucket_mb=0.0001)
    m(x).sum().backward()
    sync.wait()
    sync.remove()
    assert m[0].bias.grad is None
    for p, g in zip(m.parameters(), summed_grads(all_x)):
        if p.requires_grad:
            torch.testing.assert_close(p.grad, g)
    m[0].bias.requires_grad_(True)

    # two backwards before wait(): refused loudly (would reduce partial gradients)
    m.zero_grad(set_to_none=True)
    sync = GradSync(m, bucket_mb=64.0)  # one multi-tensor bucket
    m(x).sum().backward()
    with pytest.raises(RuntimeError, match="before wait"):
        m(x).sum().backward()
    sync.remove()

    # gradient accumulation: earlier micro-batches under no_sync(), the last one outside
    m.zero_grad(set_to_none=True)
    sync = GradSync(m, bucket_mb=0.0001)
    with sync.no_sync():
        m(x).sum().backward()
    m(2 * x).sum().backward()
    sync.wait()
    sync.remove()
    ref = summed_grads(all_x + [2 * t for t in all_x])
    for p, g in zip(m.parameters(), ref):
        torch.testing.assert_close(p.grad, g)

    # unused parameter: wait() raises by default, reduces zeros with unused='zero'
    extra = torch.nn.Linear(4, 4)
    mm = torch.nn.ModuleDict({"a": m, "b": extra})
    m.zero_grad(set_to_none=True)
    sync = GradSync(mm, bucket_mb=0.0001)
    m(x).sum().backward()
    with pytest.raises(RuntimeError, match="b.weight"):
        sync.wait()
    sync.remove()
    m.zero_grad(set_to_none=True)
    sync = GradSync(mm, bucket_mb=0.0001, unused="zero")
    m(x).sum().backward()
    sync.wait()
    sync.remove()
    assert torch.count_nonzero(extra.weight.grad) == 0
    for p, g in zip(m.parameters(), summed_grads(all_x)):
        torch.testing.assert_close(p.grad, g)

    # bf16 gradients reduced in fp32: exactly the fp32 sum rounded once
    mb = torch.nn.Linear(8, 4).to(torch.bfloat16)
    sync = GradSync(mb, bucket_mb=64.0, reduce_dtype=torch.float32)
    xb = torch.randn(5, 8, generator=torch.Generator().manual_seed(rank)).to(torch.bfloat16)
    mb(xb).float().pow(2).sum().backward()
    local = [p.grad.float().clone() for p in mb.parameters()]
    sync.wait()
    sync.remove()
    from xdot.utils import comm as C

    for p, g in zip(mb.parameters(), local):
        tot = g.clone()
        C.get_comm().all_reduce(tot, op="sum")
        assert p.grad.dtype == torch.bfloat16
        assert torch.equal(p.grad, tot.to(torch.bfloat16))


def test_gradsync_contract_gloo():
    run_gloo(_gradsync_contract_body, 2)


def _fused_delivery_body(rank, ws):
    """The fused module node hands its parameter gradients to an attached GradSync as it computes
    them (GradSync.deliver): same Sum-reduced gradients as autograd accumulation followed by
    allreduce_gradients, step by step, for two steps in a row (the second accumulates into the
    reduced .grad of the first and the bucket is reduced again: in both models the result is
    ws * G1 + sum of the step-2 local gradients)."""
    import xdot
    from xdot.parallel import GradSync, allreduce_gradients, broadcast_parameters

    torch.manual_seed(rank)
    m1 = xdot.DistributedDotProductAttn(32, num_heads=4, add_bias=True, impl="flash").double()
    broadcast_parameters(m1)
    m2 = xdot.DistributedDotProductAttn(32, num_heads=4, add_bias=True, impl="flash").double()
    m2.load_state_dict(m1.state_dict())
    sync = GradSync(m2, bucket_mb=0.0001)
    assert m2._xdot_grad_sync is not None and m1._xdot_grad_sync is None
    g = torch.Generator().manual_seed(5 + rank)
    for step in range(2):
        x = torch.rand(1, 6, 32, generator=g, dtype=torch.float64)
        m1(x, x, x, None).square().sum().backward()
        allreduce_gradients(m1)
        m2(x, x, x, None).square().sum().backward()
        sync.wait()
        for (n1, p1), (n2, p2) in zip(m1.named_parameters(), m2.named_parameters()):
            assert p2.grad is not None, n2
            torch.testing.assert_close(p2.grad, p1.grad, rtol=1e-10, atol=1e-12, msg=f"step {step} {n2}")
    sync.remove()
    assert m2._xdot_grad_sync is None


def _fused_twice_body(rank, ws):
    """One module called twice in one forward under an attached GradSync: the node must not
    deliver (the two uses are summed by AccumulateGrad first), so the reduced gradients equal the
    plain autograd + allreduce_gradients result (fused.py delivery)."""
    import xdot
    from xdot.parallel import GradSync, allreduce_gradients, broadcast_parameters

    torch.manual_seed(rank)
    m1 = xdot.DistributedDotProductAttn(32, num_heads=4, add_bias=True, impl="flash").double()
    broadcast_parameters(m1)
    m2 = xdot.DistributedDotProductAttn(32, num_heads=4, add_bias=True, impl="flash").double()
    m2.load_state_dict(m1.state_dict())
    sync = GradSync(m2, bucket_mb=0.0001)
    g = torch.Generator().manual_seed(7 + rank)
    x = torch.rand(1, 6, 32, generator=g, dtype=torch.float64)
    y = torch.rand(1, 6, 32, generator=g, dtype=torch.float64)
    for _ in range(2):  # the use count resets at wait()
        for p in list(m1.parameters()) + list(m2.parameters()):
            p.grad = None
        (m1(x, x, x, None).square().sum() + m1(y, y, y, None).pow(3).sum()).backward()
        allreduce_gradients(m1)
        (m2(x, x, x, None).square().sum() + m2(y, y, y, None).pow(3).sum()).backward()
        sync.wait()
        for (n1, p1), (n2, p2) in zip(m1.named_parameters(), m2.named_parameters()):
            torch.testing.assert_close(p2.grad, p1.grad, rtol=1e-10, atol=1e-12, msg=n2)


def _fused_frozen_body(rank, ws):
    """A frozen queries weight beside a trained values weight: the fused node hands back (and
    delivers) no gradient for the frozen one (needs_input_grad)."""
    import xdot
    from xdot.parallel import GradSync, allreduce_gradients, broadcast_parameters

    torch.manual_seed(rank)
    m1 = xdot.DistributedDotProductAttn(32, num_heads=4, add_bias=True, impl="flash").double()
    broadcast_parameters(m1)
    m2 = xdot.DistributedDotProductAttn(32, num_heads=4, add_bias=True, impl="flash").double()
    m2.load_state_dict(m1.state_dict())
    for m in (m1, m2):
        m.queries.weight.requires_grad_(False)
        m.values.bias.requires_grad_(False)
    sync = GradSync(m2, bucket_mb=0.0001)
    x = torch.rand(1, 6, 32, generator=torch.Generator().manual_seed(11 + rank), dtype=torch.float64)
    m1(x, x, x, None).square().sum().backward()
    allreduce_gradients(m1)
    m2(x, x, x, None).square().sum().backward()
    sync.wait()
    assert m2.queries.weight.grad is None and m2.values.bias.grad is None
    for (n1, p1), (n2, p2) in zip(m1.named_parameters(), m2.named_parameters()):
        if p1.requires_grad:
            torch.testing.assert_close(p2.grad, p1.grad, rtol=1e-10, atol=1e-12, msg=n2)


def _fused_no_sync_body(rank, ws):
    """Gradient accumulation with the fused module node: micro-batch 1 under no_sync(), micro-batch
    2 outside it, for two steps.  The muted backward must not mark its delivered gradients, so the
    last backward's are counted and the buckets launch (deliver() under _muted)."""
    import xdot
    from xdot.parallel import GradSync, allreduce_gradients, broadcast_parameters

    torch.manual_seed(rank)
    m1 = xdot.DistributedDotProductAttn(32, num_heads=4, add_bias=True, impl="flash").double()
    broadcast_parameters(m1)
    m2 = xdot.DistributedDotProductAttn(32, num_heads=4, add_bias=True, impl="flash").double()
    m2.load_state_dict(m1.state_dict())
    sync = GradSync(m2, bucket_mb=0.0001)
    g = torch.Generator().manual_seed(13 + rank)
    for step in range(2):
        xs = [torch.rand(1, 6, 32, generator=g, dtype=torch.float64) for _ in range(2)]
        for p in list(m1.parameters()) + list(m2.parameters()):
            p.grad = None
        for x in xs:
            m1(x, x, x, None).square().sum().backward()
        allreduce_gradients(m1)
        with sync.no_sync():
            m2(xs[0], xs[0], xs[0], None).square().sum().backward()
        m2(xs[1], xs[1], xs[1], None).square().sum().backward()
        sync.wait()
        for (n1, p1), (n2, p2) in zip(m1.named_parameters(), m2.named_parameters()):
            torch.testing.assert_close(p2.grad, p1.grad, rtol=1e-10, atol=1e-12, msg=f"step {step} {n2}")


def test_gradsync_fused_module_no_sync_accumulation():
    run_gloo(_fused_no_sync_body, 2)


def test_gradsync_fused_module_called_twice():
    run_gloo(_fused_twice_body, 2)


def test_gradsync_fused_frozen_half_of_packed_weight():
    run_gloo(_fused_frozen_body, 2)


def test_fused_module_retain_graph_twice():
    """backward twice through a retained graph of the fused module node: the second pass gives
    the same gradients again (they accumulate to twice the first), no error."""
    import xdot

    torch.manual_seed(0)
    m = xdot.DistributedDotProductAttn(32, num_heads=4, add_bias=True, impl="flash", distributed=False).double()
    x = torch.rand(1, 6, 32, dtype=torch.float64, requires_grad=True)
    loss = m(x, x, x, None).square().sum()
    loss.backward(retain_graph=True)
    g1 = [p.grad.clone() for p in m.parameters()] + [x.grad.clone()]
    loss.backward()
    g2 = [p.grad for p in m.parameters()] + [x.grad]
    for a, b in zip(g1, g2):
        torch.testing.assert_close(b, 2 * a, rtol=1e-12, atol=1e-14)


def _fused_delivery_one_step(rank, ws):
    import xdot
    from xdot.parallel import GradSync, allreduce_gradients, broadcast_parameters

    torch.manual_seed(rank)
    m1 = xdot.DistributedDotProductAttn(32, num_heads=4, add_bias=True, impl="flash").double()
    broadcast_parameters(m1)
    m2 = xdot.DistributedDotProductAttn(32, num_heads=4, add_bias=True, impl="flash").double()
    m2.load_state_dict(m1.state_dict())
    sync = GradSync(m2, bucket_mb=0.0001)
    g = torch.Generator().manual_seed(5 + rank)
    x = torch.rand(1, 6, 32, generator=g, dtype=torch.float64)
    k = torch.rand(1, 6, 32, generator=g, dtype=torch.float64)
    m1(k, x, x, None).square().sum().backward()
    m2(k, x, x, None).square().sum().backward()
    sync.wait()
    allreduce_gradients(m1)
    for (n1, p1), (n2, p2) in zip(m1.named_parameters(), m2.named_parameters()):
        torch.testing.assert_close(p2.grad, p1.grad, rtol=1e-12, atol=1e-12, msg=n1)


def test_fused_module_grad_delivery_gloo():
    run_gloo(_fused_delivery_one_step, 2)
    run_gloo(_fused_delivery_body, 2)


def test_gradsync_native_avg_matches_sum_then_divide(monkeypatch):
    """A communicator with a native average (RCCL ncclAvg: ``native_avg``) gets ONE avg collective
    per bucket and no division pass; the gradients equal the sum-then-divide route (thread ranks)."""
    from xdot.parallel import GradSync
    from xdot.utils import comm as C

    def run(native):
        monkeypatch.setattr(C.ThreadComm, "native_avg", native, raising=False)

        def body(r):
            g = torch.Generator().manual_seed(0)  # per-thread generator (threads share the global one)
            m = torch.nn.Sequential(torch.nn.Linear(6, 5), torch.nn.Linear(5, 3))
            with torch.no_grad():
                for p in m.parameters():
                    p.copy_(torch.randn(p.shape, generator=g))
            sync = GradSync(m, comm=C.get_comm(), bucket_mb=1e-5, op="avg")
            x = torch.randn(4, 6, generator=g) * (r + 1)
            m(x).square().sum().backward()
            sync.wait()
            return [p.grad.clone() for p in m.parameters()]

        return C.ThreadGroup(3).run(body)

    a, b = run(False), run(True)
    for ra, rb in zip(a, b):
        for ga, gb in zip(ra, rb):
            torch.testing.assert_close(ga, gb, rtol=1e-6, atol=1e-7)


def _wire_body(r, mode):
    """Thread rank r of test_gradsync_fp32_wire_delivery (see there)."""
    from xdot.parallel import GradSync
    from xdot.utils import comm as C

    W = C.get_comm().world_size
    m = torch.nn.Sequential(torch.nn.Linear(8, 6, bias=False), torch.nn.Linear(6, 4, bias=False)).to(torch.bfloat16)
    ps = list(m.parameters())
    sync = GradSync(m, comm=C.get_comm(), bucket_mb=1.0 if mode == "flat" else 1e-5, reduce_dtype=torch.float32)

    def g32(rank, p, salt):
        g = torch.Generator().manual_seed(100 * rank + 10 * salt + p.shape[0])
        return torch.randn(p.shape, generator=g) * (rank + 1)

    pre = {}
    if mode == "no_sync":  # a muted micro-batch first: delivered (and accumulated) in bf16
        with sync.no_sync():
            assert all(sync.wire_dtype(p) == torch.bfloat16 for p in ps)
            sync.deliver([(p, g32(r, p, 1).to(torch.bfloat16)) for p in ps])
        pre = {id(p): [g32(k, p, 1).to(torch.bfloat16).float() for k in range(W)] for p in ps}
    assert all(sync.wire_dtype(p) == torch.float32 for p in ps)
    if mode == "flat":  # one bucket: p0 on the fp32 wire, p1 in bf16 -> flattened, converted in one pass
        sync.deliver([(ps[0], g32(r, ps[0], 2)), (ps[1], g32(r, ps[1], 2).to(torch.bfloat16))])
    else:
        sync.deliver([(p, g32(r, p, 2)) for p in ps])
    sync.wait()
    for i, p in enumerate(ps):
        parts = [g32(k, p, 2) for k in range(W)]
        if mode == "flat" and i == 1:
            parts = [t.to(torch.bfloat16).float() for t in parts]
        if id(p) in pre:
            parts = [a + b for a, b in zip(parts, pre[id(p)])]
        want = sum(parts[1:], parts[0]).to(torch.bfloat16)
        assert p.grad is not None and p.grad.dtype == torch.bfloat16
        torch.testing.assert_close(p.grad, want, rtol=0, atol=0)
    return True


@pytest.mark.parametrize("mode", ["inplace", "no_sync", "flat"])
def test_gradsync_fp32_wire_delivery(mode):
    """GradSync(reduce_dtype=fp32) with bf16 parameters: a fused node hands over fp32 weight
    gradients (wire_dtype), which are all-reduced in place and written into p.grad once, rounded
    from the fp32 sum; micro-batches accumulated under no_sync() are added in fp32; a bucket that
    mixes a wire gradient with a bf16 one goes through the flat fp32 buffer.  Bitwise equal to
    rounding the fp32 sum of every rank's contribution (3 thread ranks)."""
    from xdot.utils import comm as C

    assert all(C.ThreadGroup(3).run(lambda r: _wire_body(r, mode)))


def _fused_wire_body(rank, ws):
    """bf16 fused module under GradSync(reduce_dtype=fp32): its node hands fp32 weight gradients
    over (wire_dtype) and the reduced p.grad matches an fp64 copy of the module + plain
    allreduce_gradients to bf16 accuracy, for two steps."""
    import xdot
    from xdot.parallel import GradSync, allreduce_gradients, broadcast_parameters

    torch.manual_seed(rank)
    m1 = xdot.DistributedDotProductAttn(32, num_heads=4, impl="flash").double()
    broadcast_parameters(m1)
    m2 = xdot.DistributedDotProductAttn(32, num_heads=4, impl="flash").to(torch.bfloat16)
    m2.load_state_dict({k: v.to(torch.bfloat16) for k, v in m1.state_dict().items()})
    m1.load_state_dict({k: v.to(torch.bfloat16).double() for k, v in m2.state_dict().items()})
    sync = GradSync(m2, bucket_mb=0.0001, reduce_dtype=torch.float32)
    assert all(sync.wire_dtype(p) == torch.float32 for p in m2.parameters())
    g = torch.Generator().manual_seed(17 + rank)
    for step in range(2):
        x = torch.rand(1, 8, 32, generator=g, dtype=torch.float64).to(torch.bfloat16)
        for p in list(m1.parameters()) + list(m2.parameters()):
            p.grad = None
        m1(x.double(), x.double(), x.double(), None).square().sum().backward()
        allreduce_gradients(m1)
        m2(x, x, x, None).float().square().sum().backward()
        assert len(sync._g32) == 4 and all(t.dtype == torch.float32 for t in sync._g32.values())
        sync.wait()
        for (n1, p1), (n2, p2) in zip(m1.named_parameters(), m2.named_parameters()):
            assert p2.grad is not None and p2.grad.dtype == torch.bfloat16, n2
            err = float((p2.grad.double() - p1.grad).norm() / p1.grad.norm())
            assert err < 3e-2, (step, n2, err)


def test_gradsync_fused_module_fp32_wire_gloo():
    run_gloo(_fused_wire_body, 2)


def _wire_opt_body(r):
    """Thread rank r of test_gradsync_fp32_wire_split_step_matches_plain_step."""
    from xdot.ops.optim import FusedAdamW
    from xdot.parallel import GradSync
    from xdot.utils import comm as C

    out = []
    for split in (True, False):
        m = torch.nn.Sequential(torch.nn.Linear(8, 6, bias=False), torch.nn.Linear(6, 4, bias=False)).to(torch.bfloat16)
        ps = list(m.parameters())
        gen0 = torch.Generator().manual_seed(0)  # per-thread generator (threads share the global one)
        with torch.no_grad():
            for p in ps:
                p.copy_(torch.randn(p.shape, generator=gen0))
        opt = FusedAdamW(ps, lr=1e-2)
        sync = GradSync(m, comm=C.get_comm(), bucket_mb=1e-5, reduce_dtype=torch.float32)
        for step in range(2):
            gen = torch.Generator().manual_seed(10 * r + step)
            sync.deliver([(p, torch.randn(p.shape, generator=gen)) for p in ps])
            stepped = sync.wait(optimizer=opt if split else None)
            assert stepped == split
            if not stepped:
                opt.step()
            opt.zero_grad()
        out.append([p.detach().clone() for p in ps])
    for a, b in zip(*out):  # the CPU update reads the same rounded gradient either way
        torch.testing.assert_close(a, b, rtol=0, atol=0)
    return True


def test_gradsync_fp32_wire_split_step_matches_plain_step():
    """wait(optimizer=FusedAdamW) hands the reduced fp32 gradients to the optimizer (grads=), which
    writes p.grad itself: same parameters as wait() + a plain step (3 thread ranks, CPU update)."""
    from xdot.utils import comm as C

    assert all(C.ThreadGroup(3).run(_wire_opt_body))


def test_gradsync_one_deliver_one_grouped_all_reduce(monkeypatch):
    """Buckets completed by ONE deliver() call are reduced by one grouped all-reduce (the fused
    node's end-of-backward weight gradients: one RCCL launch instead of one per bucket); values
    equal rounding the fp32 sum (3 thread ranks)."""
    from xdot.parallel import GradSync
    from xdot.utils import comm as C

    calls = {"multi": 0}
    orig_multi = C.ThreadComm.all_reduce_multi

    def multi(self, ts, op="sum", async_op=False):
        if self.rank == 0:
            calls["multi"] += 1
        return orig_multi(self, ts, op, async_op)

    monkeypatch.setattr(C.ThreadComm, "all_reduce_multi", multi)

    def body(r):
        m = torch.nn.Sequential(*[torch.nn.Linear(8, 8, bias=False) for _ in range(3)]).to(torch.bfloat16)
        ps = list(m.parameters())
        sync = GradSync(m, comm=C.get_comm(), bucket_mb=1e-5, reduce_dtype=torch.float32)
        assert len(sync.buckets) == 3
        gs = lambda rank: [torch.full(p.shape, 0.25 * (rank + 1) + i) for i, p in enumerate(ps)]
        sync.deliver(list(zip(ps, gs(r))))
        sync.wait()
        W = C.get_comm().world_size
        for i, p in enumerate(ps):
            want = sum(g[i] for g in map(gs, range(W))).to(torch.bfloat16)
            assert torch.equal(p.grad, want)
        return True

    assert all(C.ThreadGroup(3).run(body))
    assert calls["multi"] == 1
