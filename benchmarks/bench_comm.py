"""Collective micro-benchmark: all-gather and reduce-scatter of the message sizes the fused
attention moves (the bf16 [q|v] shard and its gradient partials), through the default
communicator and through the native xGMI pull collectives (``xdot.utils.ipc.IpcComm``).

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 benchmarks/bench_comm.py          # RCCL vs IPC
    torchrun --nproc-per-node 2 --master-addr 127.0.0.1 benchmarks/bench_comm.py --backend gloo   # one-GPU rehearsal

One JSON line per (collective, size, communicator) from rank 0: median µs over ``--iters``
(device-timed on the caller's stream, max over ranks) and the bus bandwidth
``(N-1)/N * bytes / t`` used by the RCCL tests.  With several ranks on ONE GPU (the gloo
rehearsal) the numbers measure the card's own HBM, not xGMI.
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--backend", default="auto", choices=["auto", "rccl", "nccl", "gloo"])
    ap.add_argument("--seq-len", type=int, default=25000, help="global T (sets the shard sizes)")
    ap.add_argument("--dim", type=int, default=768)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    a = ap.parse_args()

    from xdot.utils import comm as C
    from xdot.utils.ipc import IpcComm

    base = C.init(a.backend)
    n, rank = base.world_size, base.rank
    if n < 2:
        raise SystemExit("bench_comm needs >= 2 ranks (torchrun --nproc-per-node N)")
    dev = torch.device("cuda", C.get_local_rank() % torch.cuda.device_count())
    torch.cuda.set_device(dev)
    R = a.seq_len // n
    shapes = {  # rows x width of one rank's block
        "qv_shard_bf16": (R, 2 * a.dim),
        "qv_shard_half_bf16": (R // 2, 2 * a.dim),
        "param_bucket_bf16": (a.dim, a.dim),
    }
    comms = {base.backend: base, "ipc": IpcComm(getattr(base, "base", base))}

    def timed(fn):
        for _ in range(a.warmup):
            fn()
        ts = []
        for _ in range(a.iters):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3)
        return statistics.median(ts)

    for name, (rows, width) in shapes.items():
        x = torch.randn(rows, width, device=dev, dtype=torch.bfloat16)
        g = torch.empty(n, rows, width, device=dev, dtype=torch.bfloat16)
        parts = torch.randn(n, rows, width, device=dev, dtype=torch.bfloat16)
        out = torch.empty(rows, width, device=dev, dtype=torch.bfloat16)
        for cname, cm in comms.items():
            for coll, fn in (("all_gather", lambda: cm.all_gather_into(g, x)),
                             ("reduce_scatter", lambda: cm.reduce_scatter(out, parts))):
                us = timed(fn)
                us = max(base.all_gather_object(us))
                nbytes = n * x.numel() * x.element_size()
                if rank == 0:
                    print(json.dumps({"collective": coll, "message": name, "bytes": nbytes, "comm": cname,
                                      "world_size": n, "us": round(us, 2),
                                      "busbw_GBs": round((n - 1) / n * nbytes / us / 1e3, 2)}), flush=True)
    comms["ipc"].close()
    C.destroy()


if __name__ == "__main__":
    main()
