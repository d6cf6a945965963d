"""GEMM micro-benchmark: xdot.gemm (v1 128x128 / v2 256x256 LDS-DMA, pick with --path) vs
torch.matmul (hipBLASLt) on the distributed-product shapes (nt, all, tn) of the reference's
T=75000 / D=768 benchmarks.  Prints one JSON line per case."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters, warmup):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(iters)]
    for s, e in ev:
        s.record()
        fn()
        e.record()
    torch.cuda.synchronize()
    ts = sorted(s.elapsed_time(e) for s, e in ev)
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--cases", default="nt,all,tn,nt_small,all3,tn3")
    ap.add_argument("--path", default="auto", choices=["auto", "v1", "v2", "v3"],
                    help="xdot kernel: auto (library route for plain large products), v1 128x128, v2 256x256")
    a = ap.parse_args()
    from xdot.ops.gemm import strided_gemm

    dt = {"bf16": torch.bfloat16, "fp16": torch.float16, "fp32": torch.float32}[a.dtype]
    dev = torch.device("cuda")
    torch.manual_seed(0)
    path = a.path
    pc = {"auto": 0, "v1": 1, "v2": 2, "v3": 3}[path]
    for case in a.cases.split(","):
        if case in ("nt", "nt_small", "nt_rank8", "nt_wide") or case.startswith("ntk"):
            M = N = 75000 if case == "nt" else 25000
            K = int(case[3:]) if case.startswith("ntk") else 768
            if case == "nt_rank8":  # one rank's whole-shard nt at N=8, T=25000
                M = 3125
            if case == "nt_wide":  # 25000 x 75000 x 768 (round-2 verdict's fp32 comparison shape)
                M, N = 25000, 75000
            A = torch.randn(M, K, device=dev, dtype=dt)
            B = torch.randn(N, K, device=dev, dtype=dt)
            C = torch.empty(M, N, device=dev, dtype=dt)
            ours = lambda: strided_gemm(A, B, C, M=M, N=N, K=K, lda=K, ldb=K, ldc=N, path=pc)
            ref = lambda: torch.matmul(A, B.t(), out=C)
            flops = 2 * M * N * K
        elif case in ("all", "all3"):
            n = 1 if case == "all" else 3
            R, D = 75000 // n, 768
            T = 75000
            A = torch.randn(R, T, device=dev, dtype=dt)
            B = torch.randn(n, R, D, device=dev, dtype=dt)
            C = torch.empty(R, D, device=dev, dtype=dt)
            ours = lambda: strided_gemm(A, B, C, M=R, N=D, K=R, nseg=n, lda=T, ldb=D, ldc=D, sAseg=R,
                                        sBseg=R * D, a_mc=False, b_mc=True, path=pc)
            Bf = B.view(n * R, D)
            ref = lambda: torch.matmul(A, Bf, out=C)
            flops = 2 * R * D * T
        elif case in ("tn", "tn3"):
            n = 1 if case == "tn" else 3
            R, D = 75000 // n, 768
            T = 75000
            A = torch.randn(R, T, device=dev, dtype=dt)
            B = torch.randn(R, D, device=dev, dtype=dt)
            C = torch.empty(n, R, D, device=dev, dtype=dt)
            ours = lambda: strided_gemm(A, B, C, M=R, N=D, K=R, nb2=n, lda=T, ldb=D, ldc=D, sA2=R, sC2=R * D,
                                        a_mc=True, b_mc=True, path=pc)
            ref = lambda: torch.matmul(A.view(R, n, R).permute(1, 2, 0), B, out=C)
            flops = 2 * n * R * R * D
        elif case in ("proj", "proj_dx", "wgrad"):  # the module's projections at T = 25000, d = 768
            M, D = 25000, 768
            if case == "proj":  # y = x Wᵀ
                A = torch.randn(M, D, device=dev, dtype=dt)
                B = torch.randn(D, D, device=dev, dtype=dt)
                C = torch.empty(M, D, device=dev, dtype=dt)
                ours = lambda: strided_gemm(A, B, C, M=M, N=D, K=D, lda=D, ldb=D, ldc=D, path=pc)
                ref = lambda: torch.matmul(A, B.t(), out=C)
            elif case == "proj_dx":  # dx = dy W
                A = torch.randn(M, D, device=dev, dtype=dt)
                B = torch.randn(D, D, device=dev, dtype=dt)
                C = torch.empty(M, D, device=dev, dtype=dt)
                ours = lambda: strided_gemm(A, B, C, M=M, N=D, K=D, lda=D, ldb=D, ldc=D, b_mc=True, path=pc)
                ref = lambda: torch.matmul(A, B, out=C)
            else:  # dW = dyᵀ x (K = rows)
                A = torch.randn(M, D, device=dev, dtype=dt)
                B = torch.randn(M, D, device=dev, dtype=dt)
                C = torch.empty(D, D, device=dev, dtype=dt)
                ours = lambda: strided_gemm(A, B, C, M=D, N=D, K=M, lda=D, ldb=D, ldc=D, a_mc=True, b_mc=True, path=pc)
                ref = lambda: torch.matmul(A.t(), B, out=C)
            flops = 2 * M * D * D
        else:
            raise SystemExit(f"unknown case {case}")
        t_ours = timeit(ours, a.iters, a.warmup)
        t_ref = timeit(ref, a.iters, a.warmup)
        print(json.dumps({"case": case, "dtype": a.dtype, "path": path, "xdot_ms": round(t_ours, 3),
                          "xdot_tflops": round(flops / t_ours / 1e9, 1), "torch_ms": round(t_ref, 3),
                          "torch_tflops": round(flops / t_ref / 1e9, 1)}), flush=True)
        del A, B, C
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
