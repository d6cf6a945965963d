"""HIP-graph capture of xdot's RCCL collectives (TorchDistComm over the nccl backend): the
contract GraphedStep needs from a real communicator.  Captures all-reduce, all-gather and
reduce-scatter (after one eager warm-up call, so the communicator exists before the capture),
replays with new inputs and checks the results.  Any world size:

    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 scripts/rccl_graph_check.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    from xdot.utils import comm as C

    comm = C.init("nccl")
    n, r = comm.world_size, comm.rank
    dev = torch.device("cuda", torch.cuda.current_device())
    x = torch.zeros(1024, device=dev)
    y = torch.empty_like(x)
    gat = torch.empty(n, 1024, device=dev)
    rs = torch.empty(1024 // n if 1024 % n == 0 else 1024, device=dev)
    send = torch.empty(n * rs.numel(), device=dev)

    def body():
        y.copy_(x)
        comm.all_reduce(y, op="sum")
        comm.all_gather_into(gat, y)
        send.copy_(x.repeat(n)[: send.numel()])
        comm.reduce_scatter(rs, send)

    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):  # eager warm-up on a side stream (what GraphedStep does)
        body()
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        body()
    for it in range(3):
        x.copy_(torch.arange(1024, device=dev, dtype=torch.float32) + 1000 * r + it)
        g.replay()
        torch.cuda.synchronize()
        base = torch.arange(1024, device=dev, dtype=torch.float32) + it
        expect = n * base + 1000 * n * (n - 1) / 2
        assert torch.equal(y, expect), f"captured all-reduce, replay {it}"
        assert all(torch.equal(gat[j], expect) for j in range(n)), f"captured all-gather, replay {it}"
        k = rs.numel()
        assert torch.equal(rs, expect[r * k:(r + 1) * k] if k * n == 1024 else expect), f"captured reduce-scatter {it}"
    if r == 0:
        print("rccl-graph-ok", n, flush=True)
    C.destroy()


if __name__ == "__main__":
    main()
