"""Weight-gradient GEMM dW = dYᵀ·X (bf16 in, fp32 accumulate) at the module's shapes: xdot's
split-K MFMA path (xdot.ops.linear.weight_grad) vs hipBLASLt (torch.mm), per K = T/N rows.

    python benchmarks/bench_wgrad.py
"""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters=50):
    for _ in range(5):
        fn()
    ts = []
    for _ in range(iters):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    return statistics.median(ts)


def main():
    from xdot.ops.linear import weight_grad

    dev = torch.device("cuda", 0)
    for K in (3125, 6250, 12500, 25000):
        for M, N in ((768, 768), (1536, 768)):
            dy = torch.randn(K, M, device=dev, dtype=torch.bfloat16)
            x = torch.randn(K, N, device=dev, dtype=torch.bfloat16)
            t_x = timeit(lambda: weight_grad(dy, x))
            t_b = timeit(lambda: torch.mm(dy.t(), x))
            ref = dy.float().t() @ x.float()
            err = (weight_grad(dy, x).float() - ref).abs().max().item() / ref.abs().max().item()
            print(json.dumps({"K": K, "M": M, "N": N, "xdot_us": round(t_x, 1), "hipblaslt_us": round(t_b, 1),
                              "xdot_rel_err": err}), flush=True)


if __name__ == "__main__":
    main()
