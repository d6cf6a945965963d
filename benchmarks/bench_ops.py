"""Per-op benchmark of the distributed products, CLI-compatible with the reference.

Reference: ``benchmark.py`` (``--mode {nt,all,tn} --offset --scale --file``; 3 ranks
hard-coded; T = 75000/scale; D = 768; fp32; forward only; one cold, unsynchronised call per
process; a JSON list of 8-key records appended to ``--file``; SURVEY §3.4 / BASELINE.md).

This version keeps the CLI and the 8 record keys (``input_memory, total_time, peak_memory,
output_memory, distributed_input_memory, distributed_time, distributed_peak_memory,
distributed_output_memory``) and adds, per record:

* ``world_size``, ``T``, ``D``, ``offset``, ``dtype``, ``mode``;
* ``cold_unsynced_s`` — the reference's methodology replica (first call, ``time.time()``
  around the call, no device sync) — directly comparable to the published JSON files;
* ``ms_p50`` / ``ms_p90`` / ``ms_min`` — proper measurement: warmup, then HIP-event timing of
  ``--iters`` synchronised calls (``distributed_time`` holds the p50 in seconds).

Launch: ``python benchmarks/bench_ops.py --mode nt --scale 1`` (1 GPU) or under
``torch.distributed.run`` for N ranks.  ``--T`` overrides ``75000 // scale``.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def parse(argv=None):
    ap = argparse.ArgumentParser(description="xdot distributed op benchmark (reference-compatible)")
    ap.add_argument("--mode", default="nt", choices=["nt", "all", "tn", "rightT_fb", "full_fb", "leftT_fb"],
                    help="nt/all/tn: forward of the distributed product (reference modes); "
                         "*_fb: forward+backward of the corresponding autograd op")
    ap.add_argument("--offset", type=int, default=None, help="chunk size (default: whole shard)")
    ap.add_argument("--link-gbps", type=float, default=None,
                    help="with --emulate: collective transfer model in GB/s (xdot.utils.comm.EmulatedComm)")
    ap.add_argument("--scale", type=int, default=1, help="T = 75000 // scale (reference semantics)")
    ap.add_argument("--T", type=int, default=None)
    ap.add_argument("--dim", type=int, default=768)
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "bf16", "fp16"])
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--no-local", action="store_true", help="skip the single-GPU torch.matmul baseline")
    ap.add_argument("--file", default=None, help="JSON list to append the record to")
    ap.add_argument("--trials", type=int, default=1,
                    help="records to append (the reference's files hold 100 trials): record 0 is the "
                         "summary record above; records 1.. carry one synchronised call each "
                         "(distributed_time / total_time of that call, max over ranks)")
    ap.add_argument("--p2p-gbps", type=float, default=None, help="emulated ring-hop link rate (GB/s, --emulate)")
    ap.add_argument("--schedule", default=None, choices=["gather", "ring"],
                    help="product schedule (default XDOT_OPS_SCHEDULE / gather); also used by the *_fb modes")
    ap.add_argument("--device", default="auto", choices=["auto", "cpu"],
                    help="cpu: gloo ranks on the CPU even where a GPU is visible (BASELINE config 1)")
    ap.add_argument("--emulate", type=int, default=None, metavar="N",
                    help="run ONE rank of an N-rank job on this device (EmulatedComm: collectives are "
                         "device-local copies) -- per-rank compute of the reference's N=3 setup on 1 GPU")
    return ap.parse_args(argv)


_CUDA = [torch.cuda.is_available()]  # the timed device (False with --device cpu)


def _mem():
    return torch.cuda.memory_allocated() if _CUDA[0] else 0


def _peak_reset():
    if _CUDA[0]:
        torch.cuda.synchronize()
        torch.cuda.reset_peak_memory_stats()


def _peak():
    return torch.cuda.max_memory_allocated() if _CUDA[0] else 0


def cold_call(fn, *args):
    """Reference methodology: time.time() around one call, no device sync."""
    _peak_reset()
    m0 = _peak()
    t0 = time.time()
    y = fn(*args)
    dt = time.time() - t0
    return y, dt, _peak() - m0


def timed(fn, args, iters, warmup):
    for _ in range(warmup):
        fn(*args)
    ts = []
    for _ in range(iters):
        if _CUDA[0]:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn(*args)
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1))
        else:
            t0 = time.perf_counter()
            fn(*args)
            ts.append((time.perf_counter() - t0) * 1e3)
    raw = list(ts)
    ts.sort()
    return {"ms_p50": statistics.median(ts), "ms_p90": ts[min(len(ts) - 1, int(0.9 * len(ts)))], "ms_min": ts[0],
            "all_ms": raw}


def main(argv=None):
    a = parse(argv)
    import xdot
    from xdot.utils import comm as C
    import xdot.parallel.functional as F

    cpu = a.device == "cpu" or not torch.cuda.is_available()
    _CUDA[0] = not cpu
    comm = C.EmulatedComm(a.emulate, link_gbps=a.link_gbps, p2p_gbps=a.p2p_gbps) if a.emulate else \
        C.init("gloo" if a.device == "cpu" else "auto", set_device=not cpu)
    ctx = C.use_comm(comm)  # the functional ops pick up the thread's communicator
    ctx.__enter__()
    n, rank = comm.world_size, comm.rank
    dev = torch.device("cpu") if cpu else torch.device("cuda", C.get_local_rank() % max(1, torch.cuda.device_count()))
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
    dt = {"fp32": torch.float32, "bf16": torch.bfloat16, "fp16": torch.float16}[a.dtype]
    T = a.T or 75000 // a.scale
    T -= T % n
    R, D = T // n, a.dim
    torch.manual_seed(111)
    torch.set_grad_enabled(False)
    if a.schedule:
        from xdot.utils.env import FLAGS
        FLAGS.ops_schedule = a.schedule
    from xdot.utils.env import FLAGS as _F

    # fp32 products: which fp32 family ran (exact fp32 MFMA / library fp32 GEMM by default, the
    # reference's precision; "split" = hi/lo bf16 halves, opt-in via XDOT_FP32_MODE=split)
    fp32_mode = _F.fp32_mode if a.dtype == "fp32" else None
    # which GEMMs ran the products: the xdot kernels unless XDOT_GEMM_LIB routes them to the
    # library (csrc/bindings.cpp gemm_lib: unset / 0 = none, "fp32" = exact-fp32 ones, 1 = all)
    lib = (os.environ.get("XDOT_GEMM_LIB") or "0").strip().lower()
    on_lib = lib.startswith("1") or (lib.startswith("f") and a.dtype == "fp32")
    rec = {"mode": a.mode, "schedule": a.schedule or "gather", "world_size": n, "emulated": bool(a.emulate), "T": T, "D": D, "offset": a.offset, "dtype": a.dtype,
           "fp32_mode": fp32_mode, "link_gbps": a.link_gbps, "p2p_gbps": a.p2p_gbps,
           "gemm": "library" if on_lib else "xdot"}

    local_trials = []
    fb = a.mode.endswith("_fb")
    torch.set_grad_enabled(fb)
    # single-GPU torch baseline on the full problem (reference: rank 0 only)
    if rank == 0 and not a.no_local and not fb:
        _peak_reset()
        if a.mode == "nt":
            x = torch.rand(1, T, D, device=dev, dtype=dt)
            args = (x, x.transpose(-1, -2))
        else:
            args = (torch.rand(1, T, T, device=dev, dtype=dt), torch.rand(1, T, D, device=dev, dtype=dt))
            if a.mode == "tn":
                args = (args[0].transpose(-1, -2), args[1])
        rec["input_memory"] = _mem()
        y, t_cold, pk = cold_call(torch.matmul, *args)
        rec["total_time"] = t_cold
        rec["peak_memory"] = pk
        rec["output_memory"] = y.numel() * y.element_size()
        lt = timed(torch.matmul, args, max(3, a.iters // 2, a.trials - 1), 1)
        rec["local_" + "ms_p50"] = lt["ms_p50"]
        local_trials = lt["all_ms"]
        del args, y
        if dev.type == "cuda":
            torch.cuda.empty_cache()
    comm.barrier()

    # distributed op on this rank's shard
    if a.mode == "nt":
        left = torch.rand(1, R, D, device=dev, dtype=dt)
        right = torch.rand(1, R, D, device=dev, dtype=dt)
        fn = lambda l, r: F.distributed_matmul_nt(l, r, a.offset)  # noqa: E731
    elif a.mode == "all":
        left = torch.rand(1, R, T, device=dev, dtype=dt)
        right = torch.rand(1, R, D, device=dev, dtype=dt)
        fn = lambda l, r: F.distributed_matmul_all(l, r, a.offset)  # noqa: E731
    elif a.mode == "tn":
        left = torch.rand(1, R, T, device=dev, dtype=dt)
        right = torch.rand(1, R, D, device=dev, dtype=dt)
        fn = lambda l, r: F.distributed_matmul_tn(l, r)  # noqa: E731
    else:
        import xdot.parallel.autograd as A

        op = {"rightT_fb": A.RightTransposeMultiplication, "full_fb": A.FullMultiplication,
              "leftT_fb": A.LeftTransposeMultiplication}[a.mode]
        lshape = (1, R, D) if a.mode == "rightT_fb" else (1, R, T)
        left = torch.rand(*lshape, device=dev, dtype=dt, requires_grad=True)
        right = torch.rand(1, R, D, device=dev, dtype=dt, requires_grad=True)

        def fn(l, r):
            out = op.apply(l, r, a.offset)
            out.backward(torch.ones_like(out))
            return out.detach()
    fn.__name__ = f"distributed_{a.mode}"
    din = _mem()
    comm.barrier()
    y, t_cold, pk = cold_call(fn, left, right)
    out_mem = y.numel() * y.element_size()
    del y
    stats = timed(fn, (left, right), max(a.iters, a.trials - 1), a.warmup)
    vals = comm.all_gather_object((din, t_cold, pk, out_mem, stats))
    if rank == 0:
        avg = lambda i: sum(v[i] for v in vals) / n  # noqa: E731
        rec.update({
            "distributed_input_memory": avg(0),
            "distributed_time": max(v[4]["ms_p50"] for v in vals) / 1e3,
            "distributed_peak_memory": avg(2),
            "distributed_output_memory": avg(3),
            "cold_unsynced_s": avg(1),
            "ms_p50": max(v[4]["ms_p50"] for v in vals),
            "ms_p90": max(v[4]["ms_p90"] for v in vals),
            "ms_min": max(v[4]["ms_min"] for v in vals),
        })
        print(json.dumps(rec), flush=True)
        recs = [rec]
        for i in range(a.trials - 1):  # one record per synchronised call, in call order
            r = {k: rec[k] for k in ("mode", "schedule", "world_size", "emulated", "T", "D", "offset", "dtype", "fp32_mode", "gemm",
                                     "input_memory", "peak_memory", "output_memory", "distributed_input_memory",
                                     "distributed_peak_memory", "distributed_output_memory") if k in rec}
            r["trial"] = i + 1
            if i < len(local_trials):
                r["total_time"] = local_trials[i] / 1e3
            r["distributed_time"] = max(v[4]["all_ms"][i] for v in vals) / 1e3
            recs.append(r)
        if a.file:
            data = json.load(open(a.file)) if os.path.exists(a.file) else []
            data.extend(recs)
            json.dump(data, open(a.file, "w"), indent=1)
    comm.barrier()
    ctx.__exit__(None, None, None)
    if not a.emulate:
        C.destroy()


if __name__ == "__main__":
    main()
