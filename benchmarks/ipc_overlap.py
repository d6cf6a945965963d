"""Overlap evidence for the native xGMI pull collectives (``XDOT_IPC``): two processes share one
GPU (gloo carries the handle exchange); rank 1 joins the all-gather 20 ms late, rank 0 issues it
with ``async_op=True`` and immediately runs the attention forward of its OWN block (what the
fused path does under the gather).  Under ``rocprofv3 --kernel-trace`` the rank-0 flash kernels
sit inside the all-gather kernel's interval; the script also checks it with events: the own
block finishes while the gather is still pending.

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 benchmarks/ipc_overlap.py
"""
import json
import math
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import xdot.utils.comm as C
    from xdot.ops import flash
    from xdot.utils.ipc import IpcComm

    base = C.init("gloo")
    rank = base.rank
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    comm = IpcComm(base, capacity_mb=64, timeout_s=60)
    B, R, H, D = 1, 3125, 8, 96
    C_ = H * D
    g = torch.Generator(device=dev).manual_seed(rank)
    rows = torch.randn(B, R, C_, device=dev, dtype=torch.bfloat16, generator=g)
    qv = torch.randn(B, R, 2 * C_, device=dev, dtype=torch.bfloat16, generator=g)
    out = torch.empty(2, B, R, 2 * C_, device=dev, dtype=torch.bfloat16)
    scale = 1.0 / math.sqrt(D)
    res = []
    for it in range(4):
        base.barrier()
        torch.cuda.synchronize()
        if rank == 1:
            time.sleep(0.02)
        h = comm.all_gather_into(out, qv, async_op=True)
        e0 = torch.cuda.Event(enable_timing=True)
        e0.record()
        o, lse = flash.fwd(rows, qv[..., :C_], qv[..., C_:], None, H, scale)  # own block, no comm needed
        e1 = torch.cuda.Event(enable_timing=True)
        e1.record()
        e1.synchronize()
        pending = not h._work.is_completed() if hasattr(h, "_work") else None
        h.wait()
        torch.cuda.synchronize()
        res.append({"iter": it, "own_block_ms": round(e0.elapsed_time(e1), 3), "gather_pending_after_own_block": pending})
    comm.close()
    print(json.dumps({"rank": rank, "pid": os.getpid(), "results": res}), flush=True)
    C.destroy()


if __name__ == "__main__":
    main()
