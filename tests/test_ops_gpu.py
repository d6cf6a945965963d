"""The distributed products on the MI355X kernels with several ranks (3 gloo processes sharing
the GPU): odd rows per rank (T/N = 333, so every other column block of nt's (P, R, T) output
starts off a 16-byte boundary), offset-row chunk plans grouped per GEMM, bf16 and fp32, vs the
dense product in fp64."""
import pytest
import torch

from _dist import run_gloo

pytestmark = pytest.mark.gpu


def _ops_case(rank, ws, dt_name, offset, heads=False, schedule=None):
    import xdot.parallel.functional as F
    from xdot.utils.env import FLAGS

    if schedule is not None:
        FLAGS.ops_schedule = schedule

    dt = {"bf16": torch.bfloat16, "fp32": torch.float32}[dt_name]
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    R, D, P = 333, 96, 2
    T = R * ws
    g = torch.Generator().manual_seed(5)
    L = torch.randn(P, T, D, generator=g, dtype=torch.float64)
    Q = torch.randn(P, T, D, generator=g, dtype=torch.float64)
    S = torch.randn(P, T, T, generator=g, dtype=torch.float64) / T ** 0.5
    sl = slice(rank * R, (rank + 1) * R)
    tol = 2e-2 if dt == torch.bfloat16 else 1e-5

    def rel(a, b):
        return ((a.double() - b).norm() / b.norm()).item()

    def shard(X):  # (P, T, c) -> this rank's rows, optionally as the module's head-split view
        x = X[:, sl].to(dev, dt)
        if heads:  # (1, R, P*c) contiguous, viewed (1, P, R, c): R-major, read in place
            x = x.transpose(0, 1).contiguous().view(1, R, P, -1).transpose(1, 2)
        return x

    def flat(y):  # back to (P, R, c)
        return y.reshape(P, R, -1) if heads else y

    nt = flat(F.distributed_matmul_nt(shard(L), shard(Q), offset))
    assert rel(nt.cpu(), (L @ Q.transpose(-1, -2))[:, sl]) <= tol, "nt"
    al = flat(F.distributed_matmul_all(S[:, sl].to(dev, dt).unsqueeze(0) if heads else S[:, sl].to(dev, dt),
                                       shard(Q), offset))
    assert rel(al.cpu(), (S @ Q)[:, sl]) <= tol, "all"
    tn = flat(F.distributed_matmul_tn(S[:, sl].to(dev, dt).unsqueeze(0) if heads else S[:, sl].to(dev, dt),
                                      shard(Q)))
    assert rel(tn.cpu(), (S.transpose(-1, -2) @ Q)[:, sl]) <= tol, "tn"


@pytest.mark.parametrize("dt_name", ["bf16", "fp32"])
@pytest.mark.parametrize("offset", [32, 100, None])
@pytest.mark.parametrize("heads", [False, True])
def test_distributed_products_three_ranks(gpu, dt_name, offset, heads):
    """``heads``: operands are (1, P, R, c) head-split views of (1, R, P*c) tensors (the
    materialised module's layout): read and produced in place, no transpose copies."""
    run_gloo(_ops_case, 3, dt_name, offset, heads, timeout=300)


@pytest.mark.parametrize("dt_name", ["bf16", "fp32"])
@pytest.mark.parametrize("heads", [False, True])
def test_distributed_products_ring_schedule(gpu, dt_name, heads):
    """the same products as point-to-point ring hops (XDOT_OPS_SCHEDULE=ring): nt / all consume
    each arriving shard with one GEMM into its column block / K slice, tn's fp32 accumulators
    travel the ring; odd R = 333 and head-split views included"""
    run_gloo(_ops_case, 3, dt_name, None, heads, "ring", timeout=300)
