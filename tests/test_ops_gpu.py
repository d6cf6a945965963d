"""The distributed products on the MI355X kernels with several ranks (3 gloo processes sharing
the GPU): odd rows per rank (T/N = 333, so every other column block of nt's (P, R, T) output
starts off a 16-byte boundary), offset-row chunk plans grouped per GEMM, bf16 and fp32, vs the
dense product in fp64."""
import pytest
import torch

from _dist import run_gloo

pytestmark = pytest.mark.gpu


def _ops_case(rank, ws, dt_name, offset):
    import xdot.parallel.functional as F

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

    nt = F.distributed_matmul_nt(L[:, sl].to(dev, dt), Q[:, sl].to(dev, dt), offset)
    assert rel(nt.cpu(), (L @ Q.transpose(-1, -2))[:, sl]) <= tol, "nt"
    al = F.distributed_matmul_all(S[:, sl].to(dev, dt), Q[:, sl].to(dev, dt), offset)
    assert rel(al.cpu(), (S @ Q)[:, sl]) <= tol, "all"
    tn = F.distributed_matmul_tn(S[:, sl].to(dev, dt), Q[:, sl].to(dev, dt))
    assert rel(tn.cpu(), (S.transpose(-1, -2) @ Q)[:, sl]) <= tol, "tn"


@pytest.mark.parametrize("dt_name", ["bf16", "fp32"])
@pytest.mark.parametrize("offset", [32, 100, None])
def test_distributed_products_three_ranks(gpu, dt_name, offset):
    run_gloo(_ops_case, 3, dt_name, offset, timeout=300)
