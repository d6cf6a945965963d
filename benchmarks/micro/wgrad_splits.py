"""K-slab count of the weight-gradient kernel (csrc/gemm_wgrad.hip) per shape: GPU µs per call
(including the ordered partial sum) for S in a sweep and the launcher's automatic choice.

    python benchmarks/micro/wgrad_splits.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

import torch  # noqa: E402


def gpu_us(fn, calls=200):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(calls):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / calls * 1e3


def main():
    import argparse

    import xdot._ext as ext

    ap = argparse.ArgumentParser()
    ap.add_argument("--splits", default="0,1,2,3,4,6,8,12,16,24", help="K-slab counts (0: the launcher's choice)")
    ap.add_argument("--pair", action="store_true", help="also the paired launch of the step (dWk + dW[q|v], wgrad2)")
    args = ap.parse_args()

    assert ext.load()
    ops = ext.ops()
    dt = torch.bfloat16
    for K, M, N in [(3125, 768, 768), (3125, 1536, 768), (25000, 768, 768), (25000, 1536, 768)]:
        dy = torch.randn(K, M, device="cuda", dtype=dt)
        x = torch.randn(K, N, device="cuda", dtype=dt)
        for S in map(int, args.splits.split(",")):
            if S > (K + 63) // 64:
                continue
            us = gpu_us(lambda: ops.wgrad(dy, x, dt, S))
            print(json.dumps({"K": K, "M": M, "N": N, "S": S, "gpu_us": round(us, 2)}), flush=True)
    if args.pair:
        for K in (3125, 25000):
            a0, b0 = torch.randn(K, 768, device="cuda", dtype=dt), torch.randn(K, 768, device="cuda", dtype=dt)
            a1, b1 = torch.randn(K, 1536, device="cuda", dtype=dt), torch.randn(K, 768, device="cuda", dtype=dt)
            us = gpu_us(lambda: ops.wgrad2(a0, b0, a1, b1, dt))
            print(json.dumps({"pair_K": K, "gpu_us": round(us, 2)}), flush=True)


if __name__ == "__main__":
    main()
