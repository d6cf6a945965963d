"""A/B of the two fp32 flash families: exact fp32 MFMA (``csrc/flash_f32.hip``) vs split-bf16
(``csrc/flash_x3.hip``, 3 bf16 MFMAs per product).  One JSON line per measurement:

* ``err``: relative Frobenius error vs an fp64 reference of out / d rows / d q / d v, on the
  GPU test shapes (``tests/test_flash_gpu.CASES``, masks none / random / blocks) and at the
  headline shape (T = R = 25000, H = 8, D = 96: 32 sampled rows and columns of head 0,
  recomputed exactly in fp64);
* ``kern``: kernel times at the headline shape (fwd, bwd cols, bwd rows; median of --iters);
* ``step``: the whole bench.py training step in fp32 under each mode (N = 1).

Usage: python benchmarks/fp32_split_ab.py [--iters 5] [--steps 5]
"""
import argparse
import json
import math
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))


def rel(a, b):
    return ((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30)).item()


def case_errors(dev):
    from test_flash_f32_gpu import _inputs, _ref64
    from test_flash_gpu import CASES, _to_gathered

    from xdot.ops import flash

    for case in CASES:
        for mk_kind in ("none", "random", "blocks"):
            B, R, N, Rc, H, D = case
            T = N * Rc
            rows, kc, vc, do, mask = _inputs(case, mk_kind, dev)
            scale = 1.0 / math.sqrt(D)
            mk = flash.prepare_mask(mask, B, R, T)
            kb, vb = flash.gathered_to_btc(kc), flash.gathered_to_btc(vc)
            k, q, v, ref_o, _ = _ref64(rows, kc, vc, mask, H, scale)
            ref_o.backward(do.double())
            refs = (ref_o, k.grad.transpose(1, 2).reshape(B, R, H * D), _to_gathered(q.grad, N, B, Rc, H * D),
                    _to_gathered(v.grad, N, B, Rc, H * D))
            rec = {"kind": "err", "case": list(case), "mask": mk_kind}
            for name, fm in (("exact", 0), ("split", 1)):
                out, lse = flash.fwd(rows, kb, vb, mk, H, scale, fp32_mode=fm)
                drows, dkc, dvc = flash.bwd(do, rows, kb, vb, out, lse, mk, H, scale, fp32_mode=fm)
                got = (out, drows, flash.btc_to_rank_major(dkc, N), flash.btc_to_rank_major(dvc, N))
                rec[name] = {w: float(f"{rel(g, r):.3e}") for w, g, r in zip(("out", "drows", "dq", "dv"), got, refs)}
            print(json.dumps(rec), flush=True)


def headline(dev, iters):
    from xdot.ops import flash

    R = T = 25_000
    H, D = 8, 96
    C = H * D
    scale = 1.0 / math.sqrt(D)
    g = torch.Generator(device=dev).manual_seed(3)
    rows = torch.randn(1, R, C, device=dev, generator=g)
    kc = torch.randn(1, T, C, device=dev, generator=g)
    vc = torch.randn(1, T, C, device=dev, generator=g)
    do = torch.randn(1, R, C, device=dev, generator=g)
    ri = torch.randint(0, R, (32,), device=dev, generator=g)
    cj = torch.randint(0, T, (32,), device=dev, generator=g)
    K, V, Q, dO = kc[0, :, :D].double(), vc[0, :, :D].double(), rows[0, :, :D].double(), do[0, :, :D].double()
    s = (Q[ri] @ K.t()) * scale
    lse_r = torch.logsumexp(s, -1)
    p = torch.exp(s - lse_r[:, None])
    o_ref = p @ V
    d_ref = (dO[ri] * o_ref).sum(-1)
    dk_ref = scale * ((p * ((dO[ri] @ V.t()) - d_ref[:, None])) @ K)
    # column references need the full-row lse / δ in fp64 (recomputed chunked over rows)
    lse_all = torch.empty(R, dtype=torch.float64, device=dev)
    dl_all = torch.empty(R, dtype=torch.float64, device=dev)
    for r0 in range(0, R, 2500):
        ss = (Q[r0:r0 + 2500] @ K.t()) * scale
        l = torch.logsumexp(ss, -1)
        lse_all[r0:r0 + 2500] = l
        dl_all[r0:r0 + 2500] = (dO[r0:r0 + 2500] * (torch.exp(ss - l[:, None]) @ V)).sum(-1)
        del ss
    sc = (Q @ K[cj].t()) * scale
    pc = torch.exp(sc - lse_all[:, None])
    dsc = pc * ((dO @ V[cj].t()) - dl_all[:, None])
    dv_ref, dq_ref = pc.t() @ dO, scale * (dsc.t() @ Q)

    def timed(fn):
        ts = []
        for _ in range(iters):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            r = fn()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        ts.sort()
        return r, ts[len(ts) // 2]

    for name, fm in (("exact", 0), ("split", 1)):
        (out, lse), t_f = timed(lambda: flash.fwd(rows, kc, vc, None, H, scale, fp32_mode=fm))
        (dkv, delta), t_c = timed(lambda: flash.bwd_cols(do, rows, kc, vc, out, lse, None, H, scale, fp32_mode=fm))
        drows, t_r = timed(lambda: flash.bwd_rows(do, rows, kc, vc, lse, delta, None, H, scale, fp32_mode=fm))
        errs = {"out": rel(out[0, ri, :D], o_ref), "drows": rel(drows[0, ri, :D], dk_ref),
                "dq": rel(dkv[0, cj, :D], dq_ref), "dv": rel(dkv[0, cj, C:C + D], dv_ref)}
        flop = 4 * R * T * D * H
        print(json.dumps({"kind": "kern", "mode": name, "R": R, "T": T, "H": H, "D": D,
                          "fwd_ms": round(t_f, 3), "bwd_cols_ms": round(t_c, 3), "bwd_rows_ms": round(t_r, 3),
                          "fwd_tflops": round(flop / t_f / 1e9, 1),
                          "err_sampled": {k: float(f"{v:.3e}") for k, v in errs.items()}}), flush=True)
        del out, lse, dkv, delta, drows
        torch.cuda.empty_cache()


def step(dev, steps):
    import bench
    from xdot.utils.comm import LocalComm
    from xdot.utils.env import FLAGS

    ap = bench.parse([])
    for name in ("exact", "split"):
        FLAGS.fp32_mode = name
        ms, host_ms, lossv, impl = bench.time_step(ap, LocalComm(), dev, torch.float32, steps, 2)
        print(json.dumps({"kind": "step", "mode": name, "ms_per_step": round(ms, 3), "impl": impl,
                          "loss": lossv}), flush=True)
    FLAGS.fp32_mode = "exact"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--skip", nargs="*", default=[])
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    t0 = time.time()
    if "err" not in a.skip:
        case_errors(dev)
    if "kern" not in a.skip:
        headline(dev, a.iters)
    if "step" not in a.skip:
        step(dev, a.steps)
    print(json.dumps({"kind": "done", "s": round(time.time() - t0, 1)}), flush=True)


if __name__ == "__main__":
    main()
