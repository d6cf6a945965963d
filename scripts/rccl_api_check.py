"""RCCL code paths of xdot's TorchDistComm that gloo never reaches, run under torchrun on real
device memory: in-place all-gather (sendbuff = recvbuff + rank block), grouped all-gathers and
all-reduces (``dist._coalescing_manager``), native average, reduce-scatter, async handles, and a
GradSync round with several-gradient buckets.  Works at any world size (``tests/test_rccl_gpu.py``
runs it with one rank on the GPU box; the 8-rank node runs the same collectives).

    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 scripts/rccl_api_check.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    from xdot.parallel import GradSync
    from xdot.utils import comm as C

    be = sys.argv[1] if len(sys.argv) > 1 else "nccl"  # gloo: a CPU dry run of the same checks
    comm = C.init(be)
    n, r = comm.world_size, comm.rank
    nccl = be == "nccl"
    dev = torch.device("cuda", torch.cuda.current_device()) if nccl else torch.device("cpu")
    assert not nccl or (comm.inplace_gather and comm.native_avg), "nccl backend expected"
    # in-place all-gather: this rank's block already sits in the output
    out = torch.full((n, 4, 6), -1.0, device=dev, dtype=torch.bfloat16)
    out[r].fill_(r + 1)
    h = comm.all_gather_into(out, out[r], async_op=True)
    h.wait()
    assert all(torch.all(out[j] == j + 1) for j in range(n)), "in-place all-gather"
    # grouped chunk gathers into one buffer
    inp = torch.arange(5 * 3, device=dev, dtype=torch.float32).view(5, 3) + 100 * r
    raw = torch.empty(n * 5 * 3, device=dev)
    comm.all_gather_chunks(raw, inp, [2, 3], async_op=True).wait()
    o0 = raw[: n * 2 * 3].view(n, 2, 3)
    o1 = raw[n * 2 * 3:].view(n, 3, 3)
    for j in range(n):
        ref = torch.arange(15, device=dev, dtype=torch.float32).view(5, 3) + 100 * j
        assert torch.equal(o0[j], ref[:2]) and torch.equal(o1[j], ref[2:]), "grouped all-gather"
    # grouped in-place all-reduces, sum and avg
    ts = [torch.full((7,), float(r + 1), device=dev), torch.full((3, 2), 2.0 * (r + 1), device=dev)]
    comm.all_reduce_multi(ts, "sum", async_op=True).wait()
    tot = n * (n + 1) / 2
    assert torch.all(ts[0] == tot) and torch.all(ts[1] == 2 * tot), "grouped all-reduce"
    if comm.native_avg:
        a = torch.full((5,), float(r), device=dev)
        comm.all_reduce(a, "avg")
        assert torch.allclose(a, torch.full_like(a, (n - 1) / 2)), "native avg"
    # reduce-scatter
    send = torch.arange(n * 4, device=dev, dtype=torch.float32) * (r + 1)
    rs = torch.empty(4, device=dev)
    comm.reduce_scatter(rs, send)
    assert torch.equal(rs, torch.arange(r * 4, r * 4 + 4, device=dev, dtype=torch.float32) * tot), "reduce-scatter"
    # GradSync: one- and several-gradient buckets, avg
    torch.manual_seed(0)
    m = torch.nn.Sequential(torch.nn.Linear(16, 8), torch.nn.Linear(8, 4)).to(dev)
    sync = GradSync(m, comm=comm, bucket_mb=1e-3, op="avg")
    x = torch.randn(3, 16, device=dev)
    m(x).square().sum().backward()
    sync.wait()
    ref = torch.nn.Sequential(torch.nn.Linear(16, 8), torch.nn.Linear(8, 4)).to(dev)
    ref.load_state_dict(m.state_dict())
    ref(x).square().sum().backward()
    for p, q in zip(m.parameters(), ref.parameters()):  # identical inputs on every rank: avg == local
        torch.testing.assert_close(p.grad, q.grad)
    if nccl:
        torch.cuda.synchronize()
    if r == 0:
        print("rccl-api-ok", n, flush=True)
    C.destroy()


if __name__ == "__main__":
    main()
