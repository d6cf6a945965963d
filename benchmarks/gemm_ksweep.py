"""K sweep of the v2 NT GEMM vs torch.matmul at fixed M = N (per-item epilogue share vs K).
Prints one JSON line per K."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from benchmarks.bench_gemm import timeit  # noqa: E402


def main():
    from xdot.ops.gemm import strided_gemm
    M = int(os.environ.get("KS_M", "25000"))
    for K in (256, 768, 1536, 3072, 6144):
        A = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        B = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        C = torch.empty(M, M, device="cuda", dtype=torch.bfloat16)
        t = timeit(lambda: strided_gemm(A, B, C, M=M, N=M, K=K, lda=K, ldb=K, ldc=M), 10, 3)
        tr = timeit(lambda: torch.matmul(A, B.t(), out=C), 10, 3)
        f = 2 * M * M * K
        print(json.dumps({"M": M, "K": K, "xdot_ms": round(t, 3), "xdot_tflops": round(f / t / 1e9, 1),
                          "torch_ms": round(tr, 3), "torch_tflops": round(f / tr / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
