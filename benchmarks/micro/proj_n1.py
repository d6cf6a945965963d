"""GPU time of the N=1 (25000-row) projection GEMMs per route: the library (hipBLASLt through
torch), the projection kernel (csrc/gemm_proj.hip, forced) and the 8-phase gemm3 (path 3).

    python benchmarks/micro/proj_n1.py [--calls 50] [--rows 25000]

Shapes are the bf16 headline step's (T = 25000, d = 768; [q|v] = 1536 outputs): forward
y = x Wᵀ (NT) and input gradient dx = dy W (NN).  One JSON line per (case, route)."""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from linear_host import measure, xdot_ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=50)
    ap.add_argument("--rows", type=int, default=25000)
    ap.add_argument("--routes", default="lib,proj")
    ap.add_argument("--tiles", default="1", help="projection-kernel tile configs (xdot_gemm_proj_launch force codes)")
    args = ap.parse_args()
    from xdot.ops.gemm import strided_gemm

    ops = xdot_ops()
    dt = torch.bfloat16
    m, D = args.rows, 768
    routes = args.routes.split(",")
    cases = {"qv_fwd": ("nt", D, 2 * D), "k_fwd": ("nt", D, D), "o_dgrad": ("nn", D, D), "qv_dgrad": ("nn", 2 * D, D)}
    for name, (kind, k, n) in cases.items():
        x = torch.randn(m, k, device="cuda", dtype=dt)
        out = torch.empty(m, n, device="cuda", dtype=dt)
        res = {}
        if kind == "nt":
            w = torch.randn(n, k, device="cuda", dtype=dt) * 0.03
            ref = F.linear(x.float(), w.float())
            if "lib" in routes:
                res["lib"] = measure(lambda: F.linear(x, w), args.calls)
            if "proj" in routes:
                for t in map(int, args.tiles.split(",")):
                    res[f"proj{t}"] = measure(lambda: ops.proj(x, w, None, False, out, t, 1.0), args.calls)
                    err = float((out.float() - ref).norm() / ref.norm())
                    res[f"proj{t}"] += (err,)
            if "gemm3" in routes:
                res["gemm3"] = measure(lambda: strided_gemm(x, w, out, M=m, N=n, K=k, lda=k, ldb=k, ldc=n, path=3),
                                       args.calls)
        else:
            w = torch.randn(k, n, device="cuda", dtype=dt) * 0.03
            ref = x.float() @ w.float()
            if "lib" in routes:
                res["lib"] = measure(lambda: x @ w, args.calls)
            if "proj" in routes:
                for t in map(int, args.tiles.split(",")):
                    res[f"proj{t}"] = measure(lambda: ops.proj(x, w, None, True, out, t, 1.0), args.calls)
                    err = float((out.float() - ref).norm() / ref.norm())
                    res[f"proj{t}"] += (err,)
            if "gemm3" in routes:
                res["gemm3"] = measure(lambda: strided_gemm(x, w, out, M=m, N=n, K=k, lda=k, ldb=n, ldc=n, b_mc=True,
                                                            path=3), args.calls)
        flop = 2.0 * m * n * k
        for r, v in res.items():
            rec = {"case": name, "M": m, "N": n, "K": k, "route": r, "gpu_us": round(v[1], 2),
                   "tflops": round(flop / v[1] / 1e6, 1)}
            if len(v) > 2:
                rec["rel_err"] = v[2]
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
