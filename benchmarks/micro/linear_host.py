"""Host issue cost vs GPU time of the N=8 rank's projection GEMMs, per BLAS route.

    python benchmarks/micro/linear_host.py [--calls 200]

For each shape (T/N = 3125 rows, D = 768; [q|v] = 1536 outputs) and route, prints
  host_us   wall time to ENQUEUE one call (GPU kept busy first, so the host never waits),
  gpu_us    GPU time per call (events around `calls` calls queued behind busy work).
Routes: torch F.linear on hipBLASLt (the default), on rocBLAS ("hipblas") and CK
(`torch.backends.cuda.preferred_blas_library`), and `xdot.gemm.strided_gemm` (path 0 = xdot's
automatic kernel choice, 1 = 128x128, 2 = 256x256 v2, 3 = gemm3; the library route of the extension when XDOT_GEMM_LIB=1).
"""
from __future__ import annotations

import argparse
import json
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
    args = ap.parse_args()
    from xdot.ops.gemm import strided_gemm
    dt = torch.bfloat16
    R, D = 3125, 768
    cases = {  # name: (x rows, in, out)
        "qv_fwd": (R, D, 2 * D),
        "k_fwd": (R, D, D),
        "qv_dgrad": (R, 2 * D, D),
    }
    for name, (m, k, n) in cases.items():
        x = torch.randn(m, k, device="cuda", dtype=dt)
        w = torch.randn(n, k, device="cuda", dtype=dt) * 0.03
        b = torch.randn(n, device="cuda", dtype=dt)
        out = torch.empty(m, n, device="cuda", dtype=dt)
        res = {}
        for lib in ("hipblaslt", "hipblas", "ck"):
            torch.backends.cuda.preferred_blas_library(lib)
            res[f"torch_{lib}"] = measure(lambda: F.linear(x, w, b), args.calls)
            res[f"torch_{lib}_nobias"] = measure(lambda: F.linear(x, w), args.calls)
        torch.backends.cuda.preferred_blas_library("hipblaslt")
        for path in (0, 1, 2, 3):
            res[f"xdot_path{path}"] = measure(
                lambda: strided_gemm(x, w, out, M=m, N=n, K=k, lda=k, ldb=k, ldc=n, path=path), args.calls)
        for r, (h, g) in res.items():
            print(json.dumps({"case": name, "route": r, "host_us": round(h, 2), "gpu_us": round(g, 2)}), flush=True)


if __name__ == "__main__":
    main()
