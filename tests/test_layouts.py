"""Head-split operand layouts through the distributed products on CPU ranks:
(1, P, R, c) views of contiguous (1, R, P*c) tensors are gathered, multiplied and produced
R-major (no head-transpose / head-merge copies), with every offset plan, fp64 exact."""
import pytest
import torch


def _case(rank, ws, offset):
    import xdot.parallel.functional as F

    R, D, P = 7, 6, 3
    T = R * ws
    g = torch.Generator().manual_seed(5)
    L = torch.randn(P, T, D, generator=g, dtype=torch.float64)
    Q = torch.randn(P, T, D, generator=g, dtype=torch.float64)
    S = torch.randn(P, T, T, generator=g, dtype=torch.float64)
    sl = slice(rank * R, (rank + 1) * R)

    def shard(X):
        return X[:, sl].transpose(0, 1).contiguous().view(1, R, P, -1).transpose(1, 2)

    nt = F.distributed_matmul_nt(shard(L), shard(Q), offset)
    torch.testing.assert_close(nt.reshape(P, R, T), (L @ Q.transpose(-1, -2))[:, sl])
    al = F.distributed_matmul_all(S[:, sl].unsqueeze(0), shard(Q), offset)
    assert al.shape == (1, P, R, D) and al.transpose(1, 2).is_contiguous()  # head merge is a view
    torch.testing.assert_close(al.reshape(P, R, D), (S @ Q)[:, sl])
    tn = F.distributed_matmul_tn(S[:, sl].unsqueeze(0), shard(Q))
    assert tn.transpose(1, 2).is_contiguous()
    torch.testing.assert_close(tn.reshape(P, R, D), (S.transpose(-1, -2) @ Q)[:, sl])


@pytest.mark.parametrize("ws", [1, 3])
@pytest.mark.parametrize("offset", [2, 3, None])
def test_head_split_views(ws, offset):
    from xdot.utils.comm import ThreadGroup

    ThreadGroup(ws).run(lambda r: _case(r, ws, offset))
