"""Module-level parity: distributed fwd/bwd on shards == single-device module on full tensors.

Reference suite: ``tests/test_gradient.py`` (heads 1/4, LENGTH=18 rows per rank, DIM=256,
all-False mask, offset 32 > rows so chunking never runs, params synced by broadcast, param
grads Sum-allreduced).  Extended here: random masks (no fully-masked rows), chunked backward
(offset < rows), both execution paths ('materialized' = reference structure, 'flash' =
fused seq-parallel attention), gloo processes and in-process ranks.
"""
import pytest
import torch

from _dist import run_gloo

LENGTH = 18
DIM = 64


def _module_parity(rank, ws, heads, impl, offset, masked, dtype=torch.float64, tol=1e-9, call="kqk", bias=False,
                   length=LENGTH, batch=1):
    import xdot
    from xdot import DistributedDotProductAttn
    from xdot.parallel import broadcast_parameters, allreduce_gradients, gather_sequence

    torch.manual_seed(100 + rank)  # different init per rank: broadcast must fix it
    model = DistributedDotProductAttn(DIM, DIM, DIM, num_heads=heads, offset=offset, impl=impl,
                                      add_bias=bias).to(dtype)
    gt_model = DistributedDotProductAttn(DIM, DIM, DIM, num_heads=heads, distributed=False,
                                         impl="materialized", add_bias=bias).to(dtype)
    broadcast_parameters(model)
    gt_model.load_state_dict(model.state_dict())

    g = torch.Generator().manual_seed(7)
    T = length * ws
    k_full = torch.rand(batch, T, DIM, generator=g, dtype=dtype)
    q_full = torch.rand(batch, T, DIM, generator=g, dtype=dtype)
    if masked:
        mask_full = torch.rand(batch, T, T, generator=g) < 0.35
        mask_full[..., torch.arange(T), torch.arange(T)] = False  # no fully-masked row
    else:
        mask_full = torch.zeros(batch, T, T, dtype=torch.bool)

    sl = slice(rank * length, (rank + 1) * length)
    k = k_full[:, sl].clone().requires_grad_(True)
    q = q_full[:, sl].clone().requires_grad_(True)
    # call: which tensors go in as (keys, queries, values); "kqq" / "xxx" (queries is values) take
    # the single-node fused module path (xdot.models.fused) on the flash impl
    pick = {"kqk": lambda a, b: (a, b, a), "kqq": lambda a, b: (a, b, b), "xxx": lambda a, b: (a, a, a)}[call]
    out = model(*pick(k, q), mask_full[:, sl])
    out.sum().backward()

    kg = k_full.clone().requires_grad_(True)
    qg = q_full.clone().requires_grad_(True)
    gt_out = gt_model(*pick(kg, qg), mask_full)
    gt_out.sum().backward()

    torch.testing.assert_close(gather_sequence(out.detach(), -2), gt_out.detach(), atol=tol, rtol=tol)
    torch.testing.assert_close(gather_sequence(k.grad, -2), kg.grad, atol=tol, rtol=tol)
    if call != "xxx":
        torch.testing.assert_close(gather_sequence(q.grad, -2), qg.grad, atol=tol, rtol=tol)
    allreduce_gradients(model)
    for (n1, p1), (n2, p2) in zip(gt_model.named_parameters(), model.named_parameters()):
        assert n1 == n2
        if n1 == "queries.bias":  # exactly 0 in exact arithmetic (softmax shift invariance): noise only
            assert p2.grad.abs().max() <= 1e-6 * max(1.0, p1.grad.abs().max().item()) + 1e3 * tol
            continue
        torch.testing.assert_close(p2.grad, p1.grad, atol=tol * 10, rtol=tol * 10)


@pytest.mark.parametrize("heads", [1, 4])
@pytest.mark.parametrize("impl", ["materialized", "flash", "ring"])
def test_module_parity_gloo(heads, impl):
    run_gloo(_module_parity, 2, heads, impl, 32, True)


@pytest.mark.parametrize("ws", [1, 3])
@pytest.mark.parametrize("impl,offset", [("materialized", 5), ("materialized", None), ("flash", None),
                                         ("ring", None)])
def test_module_parity_threads(ws, impl, offset):
    from xdot.utils.comm import ThreadGroup

    ThreadGroup(ws).run(lambda r: _module_parity(r, ws, 4, impl, offset, True))


def test_module_unmasked_float32_reference_config():
    """The reference gradient-test configuration (fp32, all-False mask, atol 1e-5)."""
    from xdot.utils.comm import ThreadGroup

    ThreadGroup(2).run(lambda r: _module_parity(r, 2, 4, "materialized", 32, False,
                                                dtype=torch.float32, tol=1e-5))


@pytest.mark.parametrize("ws", [1, 3])
@pytest.mark.parametrize("call", ["kqq", "xxx"])
@pytest.mark.parametrize("fused", ["1", "0"])
def test_module_fused_node_threads(ws, call, fused, monkeypatch):
    """queries is values: the flash path runs as ONE autograd node (XDOT_FUSED_MODULE=1) or one
    node per op (0); both match the dense module (outputs, input and all 8 parameter grads)."""
    from xdot.utils.comm import ThreadGroup
    from xdot.utils.env import FLAGS

    monkeypatch.setattr(FLAGS, "fused_module", fused == "1")
    ThreadGroup(ws).run(lambda r: _module_parity(r, ws, 4, "flash", None, True, call=call, bias=True))


def test_module_fused_node_gloo():
    run_gloo(_module_parity, 2, 4, "flash", None, True, torch.float64, 1e-9, "xxx", True)
    run_gloo(_module_parity, 2, 4, "flash", None, True, torch.bfloat16, 0.08, "kqq", True)


@pytest.mark.parametrize("ws", [3, 5])
def test_ring_bidirectional_odd_rows_threads(ws):
    """Bidirectional ring with an odd row count per rank: the two lanes carry R//2 and R - R//2
    rows (exchanges of different sizes in one group), masked, with q != v inputs."""
    from xdot.utils.comm import ThreadGroup

    ThreadGroup(ws).run(lambda r: _module_parity(r, ws, 4, "ring", None, True, length=7))


@pytest.mark.parametrize("impl", ["ring", "flash"])
def test_batch_two_threads(impl):
    """B = 2: the bidirectional ring's per-lane buffers (its merged one-buffer launches are B = 1
    only) and the flash path, masked, against the dense module."""
    from xdot.utils.comm import ThreadGroup

    ThreadGroup(3).run(lambda r: _module_parity(r, 3, 4, impl, None, True, batch=2))


@pytest.mark.parametrize("ws", [3, 4])
@pytest.mark.parametrize("bidir", ["1", "0"])
def test_ring_bidirectional_gloo(ws, bidir, monkeypatch):
    """The bidirectional ring (half of every block each way, grouped two-link hops, 16-bit
    accumulators on the wire for bf16) against the dense module, fp32 and bf16, over gloo."""
    monkeypatch.setenv("XDOT_RING_BIDIR", bidir)
    run_gloo(_module_parity, ws, 4, "ring", None, True)
    run_gloo(_module_parity, ws, 4, "ring", None, True, torch.bfloat16, 0.08)


@pytest.mark.parametrize("impl", ["flash", "ring"])
def test_module_bf16_gloo(impl):
    """bf16 end to end over real gloo collectives (half-precision gathers / reductions / ring hops)."""
    run_gloo(_module_parity, 2, 4, impl, None, True, torch.bfloat16, 0.08)


def test_fully_masked_row_gives_nan():
    from xdot import DistributedDotProductAttn

    for impl in ("materialized", "flash", "ring"):
        m = DistributedDotProductAttn(16, num_heads=2, impl=impl)
        x = torch.randn(1, 4, 16)
        mask = torch.zeros(1, 4, 4, dtype=torch.bool)
        mask[0, 2] = True
        y = m(x, x, x, mask)
        assert torch.isnan(y[0, 2]).all() and not torch.isnan(y[0, 0]).any()


def test_value_dim_differs_multihead():
    """Reference raises for value_dim != key_dim with heads > 1; supported here."""
    from xdot import DistributedDotProductAttn

    m = DistributedDotProductAttn(16, value_dim=8, num_heads=2, distributed=False)
    y = m(torch.randn(1, 5, 16), torch.randn(1, 5, 16), torch.randn(1, 5, 8), None)
    assert y.shape == (1, 5, 8)


def test_state_dict_keys_match_reference():
    from xdot import DistributedDotProductAttn

    keys = set(DistributedDotProductAttn(8, num_heads=2, add_bias=True).state_dict())
    assert keys == {f"{n}.{p}" for n in ("keys", "queries", "values", "composition") for p in ("weight", "bias")}
