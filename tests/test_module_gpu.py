"""DistributedDotProductAttn on the MI355X: HIP paths vs an fp32 torch reference (GPU only).

Multi-rank cases run as separate processes sharing the one GPU (gloo transport with host
staging for the collectives): every per-rank kernel and the collective layout are the real
ones, only the wire is different from RCCL/xGMI.
"""
import pytest
import torch

from _dist import run_gloo

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12)).item()


def _module_case(rank, ws, impl, masked, dtype="bf16"):
    import xdot
    from xdot.parallel import GradSync, gather_sequence

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    torch.manual_seed(0)
    D, H, T = 256, 4, 384
    dt = {"bf16": torch.bfloat16, "fp32": torch.float32}[dtype]
    tol_o, tol_g = (2e-2, 3e-2) if dtype == "bf16" else (1e-4, 2e-4)
    m = xdot.DistributedDotProductAttn(D, num_heads=H, impl=impl, offset=None, add_bias=True).to(dev, dt)
    sync = GradSync(m, bucket_mb=0.05, reduce_dtype=torch.float32)
    g = torch.Generator(device="cpu").manual_seed(3)
    x_full = torch.randn(1, T, D, generator=g).to(dev, dt)
    mask_full = (torch.rand(1, T, T, generator=g) < 0.3) if masked else torch.zeros(1, T, T, dtype=torch.bool)
    if masked == "block":  # the first quarter of the rows sees nothing of the second half
        mask_full[:, :T // 4, T // 2:] = True    # (whole ring blocks fully masked for those rows)
    mask_full[..., torch.arange(T), torch.arange(T)] = False
    mask_full = mask_full.to(dev)
    rdt = torch.float32 if dtype == "bf16" else torch.float64
    # ground truth: plain torch ops only (no xdot kernel anywhere in the reference)
    ref = xdot.DistributedDotProductAttn(D, num_heads=H, distributed=False, impl="materialized",
                                         add_bias=True, backend="torch").to(dev, rdt)
    ref.load_state_dict({k: v.to(rdt) for k, v in m.state_dict().items()})
    xf = x_full.to(rdt).clone().requires_grad_(True)
    ref_out = ref(xf, xf, xf, mask_full)
    ref_out.pow(2).sum().backward()

    R = T // ws
    x = x_full[:, rank * R:(rank + 1) * R].clone().requires_grad_(True)
    out = m(x, x, x, mask_full[:, rank * R:(rank + 1) * R])
    assert m._pick_impl(x) == impl
    out.float().pow(2).sum().backward()
    sync.wait()  # Sum all-reduce of the replicated parameters' gradients (SP contract)
    out_all = gather_sequence(out.detach(), -2)
    gx = gather_sequence(x.grad, -2)
    assert _rel(out_all, ref_out) <= tol_o, "output"
    assert _rel(gx, xf.grad) <= tol_g, "input grad"
    names = [n for n, _ in ref.named_parameters()]
    assert len(names) == 8  # keys/queries/values/composition x (weight, bias)
    rgrad = {n: q.grad for n, q in ref.named_parameters()}
    for (n, p), (_, q) in zip(m.named_parameters(), ref.named_parameters()):
        assert p.grad is not None, n
        if n == "queries.bias":
            # exactly 0 in exact arithmetic (softmax is shift invariant along the gathered axis:
            # the bias adds k·b to a whole score row), so only rounding noise is left: bound it
            # against the same kind of row sum on the other side, the keys bias gradient
            err = (p.grad.float() - q.grad.float()).norm() / rgrad["keys.bias"].float().norm()
            assert err <= tol_g, f"grad of {n}: {err:.3e}"
            continue
        assert _rel(p.grad, q.grad) <= tol_g, f"grad of {n}: {_rel(p.grad, q.grad):.3e}"


@pytest.mark.parametrize("impl", ["materialized", "flash", "ring"])
@pytest.mark.parametrize("masked", [False, True])
def test_module_single_rank(gpu, impl, masked):
    from xdot.utils.comm import LocalComm, use_comm

    with use_comm(LocalComm()):
        _module_case(0, 1, impl, masked)


@pytest.mark.parametrize("impl", ["materialized", "flash", "ring"])
@pytest.mark.parametrize("ws", [2, 4])
def test_module_multi_rank(gpu, impl, ws):
    run_gloo(_module_case, ws, impl, True, timeout=400)


def test_module_multi_rank_unmasked_middle_ranks(gpu):
    """4 ranks, no mask: the middle ranks' gathered chunks run as ONE partial each with their own
    columns masked out by a synthetic packed mask (rank 0 / 3: one peer range, no mask)."""
    run_gloo(_module_case, 4, "flash", False, timeout=400)


@pytest.mark.parametrize("impl", ["flash", "ring"])
def test_module_multi_rank_fp32(gpu, impl):
    """fp32 on the fused paths (split-bf16 flash kernels) with 2 ranks, against an fp64 dense
    reference: the ring's per-hop split partials and fp32 accumulators included."""
    run_gloo(_module_case, 2, impl, True, "fp32", timeout=400)


@pytest.mark.parametrize("ws", [2, 4])
def test_module_ring_block_masked(gpu, ws):
    """Ring path: blocks that are fully masked for some rows (their split partials are empty)."""
    run_gloo(_module_case, ws, "ring", "block", timeout=400)


def test_flash_is_default_on_gpu_bf16(gpu):
    import xdot

    m = xdot.DistributedDotProductAttn(768, num_heads=8).to(gpu, torch.bfloat16)
    x = torch.zeros(1, 8, 768, device=gpu, dtype=torch.bfloat16)
    assert m._pick_impl(x) == "flash"


def test_module_flash_deterministic(gpu):
    """No atomics anywhere on the flash path: two identical steps are bitwise identical
    (SURVEY §5.2 determinism check)."""
    import xdot

    torch.manual_seed(0)
    m = xdot.DistributedDotProductAttn(768, num_heads=8, impl="flash").to(gpu, torch.bfloat16)
    x = torch.rand(1, 3000, 768, device=gpu, dtype=torch.bfloat16)
    mask = torch.rand(1, 3000, 3000, device=gpu) < 0.2
    mask[..., 0] = False
    res = []
    for _ in range(2):
        m.zero_grad(set_to_none=True)
        y = m(x, x, x, mask)
        y.float().square().mean().backward()
        res.append([y.detach().clone()] + [p.grad.clone() for p in m.parameters()])
    for a, b in zip(*res):
        assert torch.equal(a, b)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_module_side_stream_weight_gradients_match(gpu, dtype):
    """XDOT_WGRAD_SIDE=1 (weight gradients on side streams beside the attention backward; off by
    default) gives bitwise the same outputs and gradients as the one-stream default; in fp32 the
    library weight gradients stay on the current stream (two library GEMMs on two streams can
    stall each other: xdot.ops.linear.native_wgrad)."""
    import xdot
    from xdot.utils.env import FLAGS

    torch.manual_seed(0)
    m = xdot.DistributedDotProductAttn(768, num_heads=8, impl="flash").to(gpu, dtype)
    x = torch.rand(1, 3000, 768, device=gpu, dtype=dtype)
    res = []
    old = FLAGS.wgrad_side
    try:
        for side in (False, True):
            FLAGS.wgrad_side = side
            m.zero_grad(set_to_none=True)
            y = m(x, x, x, None)
            y.float().square().mean().backward()
            torch.cuda.synchronize()
            res.append([y.detach().clone()] + [p.grad.clone() for p in m.parameters()])
    finally:
        FLAGS.wgrad_side = old
    for a, b in zip(*res):
        assert torch.equal(a, b)


@pytest.mark.parametrize("chunks", [2, 3])
def test_module_multi_rank_gather_chunks(gpu, monkeypatch, chunks):
    """The chunked all-gather / reduce-scatter pipeline (XDOT_GATHER_CHUNKS) gives the same
    outputs and input gradients as the dense reference (2 ranks sharing the GPU over gloo)."""
    monkeypatch.setenv("XDOT_GATHER_CHUNKS", str(chunks))
    run_gloo(_module_case, 2, "flash", True, timeout=400)


def test_module_materialized_fp32_default_offset(gpu):
    """The reference configuration: fp32, default offset=32 (chunked products), materialised
    path, against an fp64 dense reference — exact-f32 MFMA GEMMs keep this at fp32 accuracy."""
    import xdot
    from xdot.utils.comm import LocalComm, use_comm

    torch.manual_seed(0)
    D, H, T = 256, 4, 200
    with use_comm(LocalComm()):
        m = xdot.DistributedDotProductAttn(D, num_heads=H, impl="materialized").to(gpu)
        assert m.offset == 32
        ref = xdot.DistributedDotProductAttn(D, num_heads=H, distributed=False, impl="materialized",
                                             backend="torch").to(gpu, torch.float64)
        ref.load_state_dict({k: v.double() for k, v in m.state_dict().items()})
        x = torch.rand(1, T, D, device=gpu, requires_grad=True)
        mask = torch.rand(1, T, T, device=gpu) < 0.3
        mask[..., 0] = False
        out = m(x, x, x, mask)
        out.pow(2).sum().backward()
        xd = x.detach().double().requires_grad_(True)
        ro = ref(xd, xd, xd, mask)
        ro.pow(2).sum().backward()
    assert _rel(out, ro) <= 1e-5
    assert _rel(x.grad, xd.grad) <= 1e-4
    for (n, p), (_, q) in zip(m.named_parameters(), ref.named_parameters()):
        assert _rel(p.grad, q.grad) <= 1e-4, n
