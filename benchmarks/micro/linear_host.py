"""Host issue cost vs GPU time of the N=8 rank's projection GEMMs, per BLAS route.

    python benchmarks/micro/linear_host.py [--calls 200]

For each shape (T/N = 3125 rows, D = 768; [q|v] = 1536 outputs) and route, prints
  host_us   wall time to ENQUEUE one call (GPU kept busy first, so the host never waits),
  gpu_us    GPU time per call (events around `calls` calls queued behind busy work).
Routes: torch F.linear / matmul on hipBLASLt (the default) and rocBLAS ("hipblas"), the projection
kernel (`torch.ops.xdot.proj`, csrc/gemm_proj.hip: forward NT and input-gradient NN; forced, and
"auto" = the op's own kernel-or-library choice), and
`xdot.gemm.strided_gemm` (path 1 = 128x128, 3 = gemm3).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.nn.functional as F


def busy(ms: float = 30.0):
    """Keep the GPU busy ~ms so enqueues never block on a full queue of finished work."""
    a = torch.randn(4096, 4096, device="cuda", dtype=torch.bfloat16)
    n = max(1, int(ms / 0.15))
    for _ in range(n):
        a = a @ a
        a = a * 1e-2
    return a


def measure(fn, calls: int):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    busy()
    t0 = time.perf_counter()
    for _ in range(calls):
        fn()
    host = (time.perf_counter() - t0) / calls * 1e6
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    busy()  # the calls queue up behind it: the events time the GPU, not the enqueue
    e0.record()
    for _ in range(calls):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return host, e0.elapsed_time(e1) / calls * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=200)
    ap.add_argument("--quick", action="store_true", help="hipBLASLt vs the projection kernel only")
    args = ap.parse_args()
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
    from xdot.ops.gemm import strided_gemm
    dt = torch.bfloat16
    R, D = 3125, 768
    ops = xdot_ops()
    cases = {  # name: (kind, rows, in, out); nt = forward x Wᵀ + b, nn = input gradient dy W
        "qv_fwd": ("nt", R, D, 2 * D),
        "k_fwd": ("nt", R, D, D),
        "qv_dgrad": ("nn", R, 2 * D, D),
        "k_dgrad": ("nn", R, D, D),
        "qv_fwd_n4": ("nt", 2 * R, D, 2 * D),
        "qv_dgrad_n4": ("nn", 2 * R, 2 * D, D),
        "qv_fwd_n2": ("nt", 4 * R, D, 2 * D),
        "qv_fwd_n1": ("nt", 8 * R, D, 2 * D),
        "qv_dgrad_n1": ("nn", 8 * R, 2 * D, D),
    }
    for name, (kind, m, k, n) in cases.items():
        x = torch.randn(m, k, device="cuda", dtype=dt)
        res = {}
        if kind == "nt":
            w = torch.randn(n, k, device="cuda", dtype=dt) * 0.03
            b = torch.randn(n, device="cuda", dtype=dt)
            out = torch.empty(m, n, device="cuda", dtype=dt)
            for lib in ("hipblaslt", "hipblas") if not args.quick else ("hipblaslt",):
                torch.backends.cuda.preferred_blas_library(lib)
                res[f"torch_{lib}"] = measure(lambda: F.linear(x, w, b), args.calls)
                res[f"torch_{lib}_nobias"] = measure(lambda: F.linear(x, w), args.calls)
            torch.backends.cuda.preferred_blas_library("hipblaslt")
            res["xdot_proj"] = measure(lambda: ops.proj(x, w, b, False, None, 1), args.calls)
            res["xdot_proj_nobias"] = measure(lambda: ops.proj(x, w, None, False, None, 1), args.calls)
            res["xdot_proj_auto"] = measure(lambda: ops.proj(x, w, b, False, None, 0), args.calls)
            for path in (1, 3) if not args.quick else ():
                res[f"xdot_path{path}"] = measure(
                    lambda: strided_gemm(x, w, out, M=m, N=n, K=k, lda=k, ldb=k, ldc=n, path=path), args.calls)
        else:
            w = torch.randn(k, n, device="cuda", dtype=dt) * 0.03  # Linear(n -> k) weight: dx = dy W
            res["torch_hipblaslt"] = measure(lambda: x @ w, args.calls)
            res["xdot_proj"] = measure(lambda: ops.proj(x, w, None, True, None, 1), args.calls)
            res["xdot_proj_auto"] = measure(lambda: ops.proj(x, w, None, True, None, 0), args.calls)
        for r, (h, g) in res.items():
            print(json.dumps({"case": name, "M": m, "N": n, "K": k, "route": r, "host_us": round(h, 2),
                              "gpu_us": round(g, 2)}), flush=True)
    wgrad_cases(args, dt, ops)


def wgrad_cases(args, dt, ops):
    """Weight gradients dyᵀ·x (K = rows): hipBLASLt vs the gemm3 split-K route vs
    csrc/gemm_wgrad.hip (each including its partial reduction)."""
    from xdot.ops.gemm import strided_gemm

    for name, (K, M, N) in {"wk_rank8": (3125, 768, 768), "wqv_rank8": (3125, 1536, 768),
                            "wk_n1": (25000, 768, 768), "wqv_n1": (25000, 1536, 768)}.items():
        dy = torch.randn(K, M, device="cuda", dtype=dt)
        x = torch.randn(K, N, device="cuda", dtype=dt)
        out = torch.empty(M, N, device="cuda", dtype=dt)
        res = {"torch_hipblaslt": measure(lambda: (dy.t() @ x), args.calls),
               "xdot_gemm3_splitk": measure(lambda: strided_gemm(dy, x, out, M=M, N=N, K=K, lda=M, ldb=N, ldc=N,
                                                                 a_mc=True, b_mc=True, path=5), args.calls),
               "xdot_wgrad": measure(lambda: ops.wgrad(dy, x, dt, 0), args.calls)}
        for r, (h, g) in res.items():
            print(json.dumps({"case": name, "M": M, "N": N, "K": K, "route": r, "host_us": round(h, 2),
                              "gpu_us": round(g, 2)}), flush=True)


def xdot_ops():
    import xdot._ext as ext

    assert ext.load(), "xdot/_C.so missing"
    return ext.ops()


if __name__ == "__main__":
    main()
