"""Kernel-level timing of the flash-attention kernels at the headline shape (per rank).

    python benchmarks/bench_flash.py                       # T=25000, R=25000 (N=1), H=8, D=96
    python benchmarks/bench_flash.py --R 3125              # the per-rank shape at N=8
    python benchmarks/bench_flash.py --only fwd --iters 20 # (for rocprofv3 --pmc runs)

Prints one JSON line per kernel: median ms over ``--iters`` HIP-event timed calls and the
achieved TFLOP/s (fwd: 2 GEMMs, bwd_rows: 3, bwd_cols: 4; 2*R*T*H*D FLOP each), plus the
materialised reference path (torch SDPA math on the same shape) when ``--torch`` is given.
"""
import argparse
import json
import math
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters, warmup=2):
    for _ in range(warmup):
        fn()
    ts = []
    for _ in range(iters):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1))
    return statistics.median(ts), min(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--T", type=int, default=25000)
    ap.add_argument("--R", type=int, default=None)
    ap.add_argument("--H", type=int, default=8)
    ap.add_argument("--D", type=int, default=96)
    ap.add_argument("--B", type=int, default=1)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--only", default="all", choices=["all", "fwd", "bwd_cols", "bwd_rows", "mask"])
    ap.add_argument("--mask", action="store_true", help="pass an all-False (B, R, T) mask")
    ap.add_argument("--mask-density", type=float, default=0.0,
                    help="with --mask: fraction of randomly masked entries (0: all-False)")
    ap.add_argument("--nsplit", type=int, default=0)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp16", "fp32"])
    ap.add_argument("--fp32-mode", default=None, choices=["split", "exact"],
                    help="fp32 kernel family (default: XDOT_FP32_MODE)")
    ap.add_argument("--no-prescale", action="store_true",
                    help="kernels scale every score (default: pre-scaled rows + seeded accumulators, the module's path)")
    ap.add_argument("--scores", action="store_true",
                    help="fp32 (exact or split): score-buffer mode (forward stores S, bwd_cols reads S and writes dS, "
                         "bwd_rows reads dS; products 2 / 3 / 1 instead of 2 / 4 / 3)")
    ap.add_argument("--torch", action="store_true", help="also time torch SDPA (aotriton) on the same shape")
    ap.add_argument("--concurrent", action="store_true",
                    help="also time bwd_cols and bwd_rows launched together on two streams (cols on a normal "
                         "and on a high-priority stream): when cols finishes and when both finish")
    a = ap.parse_args()
    from xdot.ops import flash

    dev = torch.device("cuda", 0)
    B, T, H, D = a.B, a.T, a.H, a.D
    R = a.R or T
    C = H * D
    g = torch.Generator(device=dev).manual_seed(0)
    dt = {"bf16": torch.bfloat16, "fp16": torch.float16, "fp32": torch.float32}[a.dtype]
    if a.fp32_mode is not None:
        from xdot.utils.env import FLAGS

        FLAGS.fp32_mode = a.fp32_mode
    rows = torch.randn(B, R, C, device=dev, dtype=dt, generator=g)
    qv = torch.randn(B, T, 2 * C, device=dev, dtype=dt, generator=g)
    kc, vc = qv[..., :C], qv[..., C:]
    do = torch.randn(B, R, C, device=dev, dtype=dt, generator=g)
    mask = None
    if a.mask:
        mask = torch.rand(B, R, T, device=dev, generator=g) < a.mask_density
        mask[..., 0] = False
    mk = flash.prepare_mask(mask, B, R, T)
    scale = 1.0 / math.sqrt(D)
    ps = not a.no_prescale and dt != torch.float32
    rk = flash.prescale(rows, scale) if ps else rows
    sb = None
    if a.scores:
        assert dt == torch.float32, "--scores is an fp32 (exact or split) mode"
        sb = flash.score_buffer(B, H, R, T, dev)
        assert sb is not None, "score buffer does not fit"
    # (timing only: after the first bwd_cols the buffer holds dS, which later calls read as S)
    out, lse = flash.fwd(rk, kc, vc, mk, H, scale, a.nsplit, prescaled=ps, sbuf=sb)
    # score-buffer mode: the fused exact column pass where the module uses it (XDOT_F32_FUSED_COLS)
    cpasses = 4 if sb is not None and flash.fused_cols_wanted(flash.fp32_code(dt), D) else 3
    dkv, delta = flash.bwd_cols(do, rk, kc, vc, out, lse, mk, H, scale, prescaled=ps, sbuf=sb, passes=cpasses)
    gemm = 2.0 * B * R * T * H * D
    np_cols, np_rows = (3, 1) if sb is not None else (4, 3)
    res = []
    if a.only in ("all", "mask") and mask is not None:
        ms, mn = timeit(lambda: flash.prepare_mask(mask, B, R, T), a.iters)
        res.append({"kernel": "mask_pack", "ms": ms, "min_ms": mn, "GB_s": B * R * T / ms / 1e6})
    if a.only in ("all", "fwd"):
        ms, mn = timeit(lambda: flash.fwd(rk, kc, vc, mk, H, scale, a.nsplit, prescaled=ps, sbuf=sb), a.iters)
        res.append({"kernel": "flash_fwd" + ("+S" if sb is not None else ""), "ms": ms, "min_ms": mn,
                    "TFLOPs": 2 * gemm / ms / 1e9})
    if a.only in ("all", "bwd_cols"):
        ms, mn = timeit(lambda: flash.bwd_cols(do, rk, kc, vc, out, lse, mk, H, scale, prescaled=ps, sbuf=sb,
                                               passes=cpasses), a.iters)
        res.append({"kernel": "flash_bwd_cols" + ("(S->dS)" if sb is not None else ""), "ms": ms, "min_ms": mn,
                    "TFLOPs": np_cols * gemm / ms / 1e9})
    if a.only in ("all", "bwd_rows"):
        ms, mn = timeit(lambda: flash.bwd_rows(do, rk, kc, vc, lse, delta, mk, H, scale, a.nsplit, prescaled=ps,
                                               sbuf=sb), a.iters)
        res.append({"kernel": "flash_bwd_rows" + ("(dS)" if sb is not None else ""), "ms": ms, "min_ms": mn,
                    "TFLOPs": np_rows * gemm / ms / 1e9})
    if a.concurrent:
        for prio in (0, -1):
            side = torch.cuda.Stream(device=dev, priority=prio)
            cur = torch.cuda.current_stream(dev)
            tc, tb = [], []
            for it in range(a.iters + 2):
                e0, ec, e1 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
                e0.record()
                side.wait_stream(cur)
                with torch.cuda.stream(side):
                    flash.bwd_cols(do, rk, kc, vc, out, lse, mk, H, scale, delta, prescaled=ps)
                    ec.record()
                flash.bwd_rows(do, rk, kc, vc, lse, delta, mk, H, scale, a.nsplit, prescaled=ps)
                cur.wait_stream(side)
                e1.record()
                e1.synchronize()
                if it >= 2:
                    tc.append(e0.elapsed_time(ec))
                    tb.append(e0.elapsed_time(e1))
            res.append({"kernel": f"cols||rows prio={prio}", "ms": statistics.median(tb),
                        "cols_done_ms": statistics.median(tc), "min_ms": min(tb)})
    if a.torch and R == T:
        q = rows.view(B, R, H, D).transpose(1, 2).contiguous().requires_grad_(True)
        k = kc.reshape(B, T, H, D).transpose(1, 2).contiguous().requires_grad_(True)
        v = vc.reshape(B, T, H, D).transpose(1, 2).contiguous().requires_grad_(True)
        f = lambda: torch.nn.functional.scaled_dot_product_attention(q, k, v)  # noqa: E731
        ms, mn = timeit(f, a.iters)
        res.append({"kernel": "torch_sdpa_fwd", "ms": ms, "min_ms": mn, "TFLOPs": 2 * gemm / ms / 1e9})
        o = f()
        gout = torch.randn_like(o)
        ms, mn = timeit(lambda: torch.autograd.grad(f(), (q, k, v), gout), a.iters)
        res.append({"kernel": "torch_sdpa_fwd+bwd", "ms": ms, "min_ms": mn, "TFLOPs": 7 * gemm / ms / 1e9})
    for r in res:
        r.update({"B": B, "R": R, "T": T, "H": H, "D": D})
        print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in r.items()}))


if __name__ == "__main__":
    main()
