"""Headline benchmark: DistributedDotProductAttn training step, T=25000, d=768, h=8.

Metric (BASELINE.json): ``ms/fwd+bwd DistributedDotProductAttn T=25000 d=768 h=8; scaling
1/2/4/8 GPU``.  One step = forward + backward of the module on this rank's T/N rows
(global T fixed => strong scaling), MSE loss as in the reference ``example.py``, the
sequence-parallel Sum all-reduce of the replicated parameter gradients and an AdamW step.
Synthetic random inputs, random-init weights, bf16 compute, the reference's all-False
boolean mask (``example.py:29``) is passed and honoured.

    python bench.py --gpus 1 --steps 10 --warmup 3
    python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
        --master-port 29500 bench.py --gpus 8 --steps 20 --warmup 5

Rank 0 prints one JSON line.  ``value`` = wall ms per step, max over ranks (the job's step
time); the timed region is bracketed by a barrier and ``torch.cuda.synchronize()``.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

# kernel arguments in device memory: lower launch latency for the step's ~26 launches (read by
# the HIP runtime at its initialisation, i.e. before the first GPU call).  Same-box A/B, 3 rounds:
# N=1 7.90 -> 7.86 ms, emulated N=8 rank 1.339 -> 1.306 ms (profiles/r2_kernarg.md)
os.environ.setdefault("HIP_FORCE_DEV_KERNARG", "1")

import torch  # noqa: E402

METRIC = "ms/fwd+bwd DistributedDotProductAttn T=25000 d=768 h=8; scaling 1/2/4/8 GPU"


def parse(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--seq-len", type=int, default=25000, help="global T")
    ap.add_argument("--dim", type=int, default=768)
    ap.add_argument("--heads", type=int, default=8)
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp16", "fp32"])
    ap.add_argument("--impl", default="auto", choices=["auto", "flash", "materialized", "ring"])
    ap.add_argument("--offset", type=int, default=None)
    ap.add_argument("--mask", default="zeros", choices=["zeros", "none", "random"])
    ap.add_argument("--no-optim", action="store_true", help="(diagnostic) skip the optimizer step")
    ap.add_argument("--optim", default="xdot", choices=["xdot", "torch"],
                    help="AdamW implementation: xdot.FusedAdamW (one HIP launch) or torch's fused AdamW")
    ap.add_argument("--device", default="cuda")
    ap.add_argument("--backend", default="auto", choices=["auto", "rccl", "nccl", "gloo"],
                    help="collective backend (auto = RCCL on GPU); gloo lets several ranks share one GPU "
                         "for rehearsals")
    ap.add_argument("--profile-dir", default=None, help="write a torch.profiler trace here")
    ap.add_argument("--no-split-step", dest="split_step", action="store_false",
                    help="(A/B) one optimizer step after every all-reduce instead of splitting it around the last one")
    ap.add_argument("--graph", action="store_true",
                    help="capture the whole step (fwd+bwd+grad sync+AdamW) in a HIP graph and replay it "
                         "(xdot.utils.graphs.GraphedStep; single-GPU / emulated communicators)")
    return ap.parse_args(argv)


def main(argv=None, comm=None):
    """``comm``: optional communicator override (``benchmarks/bench_rank.py`` passes an
    :class:`xdot.utils.comm.EmulatedComm` to run one rank of an N-GPU step on one GPU)."""
    a = parse(argv)
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import xdot
    from xdot.utils import comm as C
    from xdot.parallel import GradSync

    emulated = comm is not None
    comm = comm or C.init(a.backend)
    n, rank = comm.world_size, comm.rank
    if n != a.gpus and rank == 0:
        print(f"warning: --gpus {a.gpus} but world size {n}", file=sys.stderr)
    dev = torch.device(a.device, C.get_local_rank() % max(1, torch.cuda.device_count())) if a.device == "cuda" \
        else torch.device("cpu")
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
    dt = {"bf16": torch.bfloat16, "fp16": torch.float16, "fp32": torch.float32}[a.dtype]
    T = a.seq_len
    if T % n:
        raise SystemExit(f"seq-len {T} not divisible by world size {n}")
    R = T // n

    torch.manual_seed(1234)  # identical weights on every rank
    model = xdot.DistributedDotProductAttn(a.dim, num_heads=a.heads, offset=a.offset, impl=a.impl,
                                        comm=comm).to(dev, dt)
    if a.optim == "xdot":
        # one multi-tensor HIP launch per step (device-side step count when graph-captured)
        opt = xdot.FusedAdamW(model.parameters(), lr=1e-4, capturable=a.graph)
    else:
        opt = torch.optim.AdamW(model.parameters(), lr=1e-4, fused=(dev.type == "cuda"))
    sync = GradSync(model, comm=comm, bucket_mb=1.0)  # per-parameter buckets: the output
    # projection's all-reduce overlaps the attention backward
    crit = xdot.MSELoss()  # fused loss + gradient pass (torch.nn.MSELoss semantics)
    from xdot.ops.loss import unit_grad

    g = torch.Generator(device=dev).manual_seed(1000 + rank)
    x = torch.rand(a.batch, R, a.dim, device=dev, dtype=dt, generator=g)
    y = torch.rand(a.batch, R, a.dim, device=dev, dtype=dt, generator=g)
    if a.mask == "none":
        mask = None
    elif a.mask == "zeros":
        mask = torch.zeros(a.batch, R, T, dtype=torch.bool, device=dev)
    else:
        mask = torch.rand(a.batch, R, T, device=dev, generator=g) < 0.1
        mask[..., 0] = False

    def step():
        opt.zero_grad(set_to_none=True)
        out = model(x, x, x, mask)
        loss = crit(out, y)
        loss.backward(unit_grad(loss))  # == loss.backward(), minus the seed fill / scaling pass
        # with several ranks the update of the buckets already reduced runs under the last
        # gradient all-reduce (GradSync.wait(optimizer=...)); otherwise one step after the wait
        stepped = sync.wait(optimizer=None if a.no_optim or not a.split_step else opt)
        if not a.no_optim and not stepped:
            opt.step()
        return loss

    if a.graph:
        from xdot.utils.graphs import GraphedStep

        def body():
            out = model(x, x, x, mask)
            loss = crit(out, y)
            loss.backward()
            sync.wait()
            if not a.no_optim:
                opt.step()
            return loss

        step = GraphedStep(body, zero_grad=opt.zero_grad, warmup=max(1, a.warmup))
        step()  # warmup steps + capture + one replay
    else:
        for _ in range(a.warmup):
            step()
    impl = model._pick_impl(x)

    def sync_all():
        if dev.type == "cuda":
            torch.cuda.synchronize()
        comm.barrier()

    prof = None
    if a.profile_dir and rank == 0:
        prof = torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU,
                                                  torch.profiler.ProfilerActivity.CUDA])
        prof.__enter__()
    sync_all()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        loss = step()
    th = time.perf_counter()  # host done enqueuing (diagnostic: close to t1 = host-bound step)
    sync_all()
    t1 = time.perf_counter()
    if prof is not None:
        prof.__exit__(None, None, None)
        os.makedirs(a.profile_dir, exist_ok=True)
        prof.export_chrome_trace(os.path.join(a.profile_dir, "trace.json"))
        with open(os.path.join(a.profile_dir, "ops.txt"), "w") as f:
            f.write(prof.key_averages().table(sort_by="cuda_time_total", row_limit=40))

    ms = (t1 - t0) * 1e3 / max(1, a.steps)
    t = torch.tensor([ms], dtype=torch.float64, device=dev if comm.backend in ("nccl", "emulated") else "cpu")
    comm.all_reduce(t, op="max")
    ms = float(t.item())
    lossv = float(loss.float().item())
    if not math.isfinite(lossv):
        raise SystemExit(f"non-finite loss {lossv}")
    if rank == 0:
        metric = METRIC
        if (T, a.dim, a.heads) != (25000, 768, 8):  # not the headline config: say what was run
            metric = f"ms/fwd+bwd DistributedDotProductAttn T={T} d={a.dim} h={a.heads}"
        rec = {
            "metric": metric,
            "value": round(ms, 4),
            "unit": "ms",
            "n_gpus": n,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms, 4),
            "higher_is_better": False,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": a.dtype,
            "data": "synthetic (random inputs, random-init weights)",
            "config": {"model": f"DistributedDotProductAttn(d={a.dim},h={a.heads})", "global_batch": a.batch,
                       "seq_len": T, "parallelism": f"sp{n}", "impl": impl, "mask": a.mask,
                       "step": "fwd+bwd+grad-allreduce+AdamW" if not a.no_optim else "fwd+bwd+grad-allreduce",
                       "launch": "hip-graph" if a.graph else "eager"},
            "tokens_per_s": round(a.batch * T / (ms / 1e3), 1),
            "host_enqueue_ms_per_step": round((th - t0) * 1e3 / max(1, a.steps), 4),
            "loss": lossv,
        }
        if emulated:
            link = getattr(comm, "link_gbps", None)
            what = "no transport" if link is None else f"link model {link:g} GB/s collectives, {comm.p2p_gbps:g} GB/s hops"
            rec["metric"] = f"EMULATED per-rank step ({what}; diagnostics only): " + metric
            rec["config"]["parallelism"] += "-emulated"
        print(json.dumps(rec), flush=True)
    if not emulated:
        C.destroy()
    return ms


if __name__ == "__main__":
    main()
