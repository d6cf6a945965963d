"""Headline benchmark: DistributedDotProductAttn training step, T=25000, d=768, h=8.

Metric (BASELINE.json): ``ms/fwd+bwd DistributedDotProductAttn T=25000 d=768 h=8; scaling
1/2/4/8 GPU``.  One step = forward + backward of the module on this rank's T/N rows
(global T fixed => strong scaling), MSE loss as in the reference ``example.py``, the
sequence-parallel Sum all-reduce of the replicated parameter gradients and an AdamW step.
Synthetic random inputs, random-init weights, bf16 compute, the reference's all-False
boolean mask (``example.py:29``) is passed and honoured.

    python bench.py --gpus 1 --steps 10 --warmup 3
    python bench.py --gpus 8 --steps 20 --warmup 5        # starts the 8-rank torchrun job itself
    python bench.py --sweep 1,2,4,8                        # one line per N + a scaling summary
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
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks (one per GPU).  Without a launcher in the environment, N > 1 starts the "
                         "N-rank torchrun job itself")
    ap.add_argument("--sweep", default=None,
                    help="comma-separated N list (e.g. 1,2,4,8): run each N in fresh processes, print one "
                         "JSON line per N and a speed-up / efficiency summary line")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=10,
                    help="untimed steps first (10: about 1 %% faster timed steps than 3 on the same box, scripts/archive/warm_ab.sh)")
    ap.add_argument("--seq-len", type=int, default=25000, help="global T")
    ap.add_argument("--dim", type=int, default=768)
    ap.add_argument("--heads", type=int, default=8)
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp16", "fp32"])
    ap.add_argument("--impl", default="auto", choices=["auto", "flash", "materialized", "ring"])
    ap.add_argument("--offset", type=int, default=None)
    ap.add_argument("--mask", default="zeros", choices=["zeros", "none", "random", "block-causal"],
                    help="zeros: the reference example's all-False mask (example.py:29); random: 10 %% masked; "
                         "block-causal: 1024-wide causal blocks")
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
    ap.add_argument("--no-check", action="store_true",
                    help="skip the T=512 numerics check of the N-rank module against the dense fp32 module")
    ap.add_argument("--fp32-steps", type=int, default=5,
                    help="also time this many steps of the same step in fp32 (the reference's precision; "
                         "0 = skip); reported as fp32_ms_per_step")
    ap.add_argument("--fp32-warmup", type=int, default=2)
    ap.add_argument("--no-diagnostics", dest="diagnostics", action="store_false",
                    help="N > 1: skip the post-timing breakdown (collectives alone, compute-only step)")
    ap.add_argument("--trace", action="store_true",
                    help="print stage / step progress with timestamps to stderr (diagnostics)")
    ap.add_argument("--graph", action="store_true",
                    help="capture the whole step (fwd+bwd+grad sync+AdamW) in a HIP graph and replay it "
                         "(xdot.utils.graphs.GraphedStep; single-GPU / emulated communicators)")
    return ap.parse_args(argv)


_T0 = time.perf_counter()


def _trace(a, msg):
    if getattr(a, "trace", False):
        print(f"[bench {time.perf_counter() - _T0:8.2f}s] {msg}", file=sys.stderr, flush=True)


def numerics_check(a, comm, dev, dt, impl, T: int = 512, tol: float = 3e-2) -> float:
    """Before timing: a T=512 forward+backward of the module on THIS job's ranks (same
    communicator, impl and dtype as the timed step, a random 10 % mask) against the dense
    single-device fp32 module (``distributed=False``) on the full sequence, which every rank
    recomputes (the reference's test_gradient.py pattern).  Compares this rank's output rows,
    input gradient and the Sum-all-reduced parameter gradients (relative Frobenius); raises
    SystemExit(3) on a mismatch.  Returns the worst relative error."""
    import xdot
    from xdot.parallel import allreduce_gradients

    n, rank = comm.world_size, comm.rank
    T = max(T // n, 1) * n
    R = T // n
    torch.manual_seed(4321)  # identical weights on every rank
    m = xdot.DistributedDotProductAttn(a.dim, num_heads=a.heads, impl=impl, comm=comm).to(dev, dt)
    ref = xdot.DistributedDotProductAttn(a.dim, num_heads=a.heads, distributed=False, impl="materialized",
                                         backend="torch").to(dev, torch.float32)  # plain torch ops
    ref.load_state_dict({k: v.float() for k, v in m.state_dict().items()})
    g = torch.Generator(device=dev).manual_seed(99)  # identical full inputs on every rank
    xf = torch.rand(1, T, a.dim, device=dev, generator=g)
    mask = torch.rand(1, T, T, device=dev, generator=g) < 0.1
    mask[..., 0] = False
    rows = slice(rank * R, (rank + 1) * R)
    x = xf[:, rows].to(dt).requires_grad_(True)
    out = m(x, x, x, mask[:, rows].contiguous())
    (out.float().square().sum() / (T * a.dim)).backward()
    allreduce_gradients(m, comm=comm)  # per-rank partial parameter grads -> their sum
    xr = xf.clone().requires_grad_(True)
    outr = ref(xr, xr, xr, mask)
    (outr.square().sum() / (T * a.dim)).backward()

    def rel(u, v):
        return float((u.detach().float() - v.detach().float()).norm() / v.detach().float().norm().clamp_min(1e-30))

    errs = {"out": rel(out, outr[:, rows]), "dx": rel(x.grad, xr.grad[:, rows])}
    for (name, p), (_, pr) in zip(m.named_parameters(), ref.named_parameters()):
        errs["d" + name] = rel(p.grad, pr.grad)
    worst = max(errs.values())
    t = torch.tensor([worst], dtype=torch.float64, device=dev if "gloo" not in comm.backend else "cpu")
    comm.all_reduce(t, op="max")
    worst = float(t.item())
    if not worst <= tol:  # NaN fails too
        raise SystemExit(f"bench numerics check failed on rank {rank} (N={n}, T={T}, {impl}, {dt}): {errs}")
    return worst


def time_step(a, comm, dev, dt, steps, warmup, graph=False, profile_dir=None):
    """Build the model/optimizer for ``dt`` and time ``steps`` training steps after
    ``warmup`` untimed ones.  Returns (ms_per_step max over ranks, host enqueue ms, loss, impl)."""
    import xdot
    from xdot.parallel import GradSync
    from xdot.ops.loss import backward, unit_grad

    n, rank = comm.world_size, comm.rank
    T = a.seq_len
    R = T // n
    torch.manual_seed(1234)  # identical weights on every rank
    model = xdot.DistributedDotProductAttn(a.dim, num_heads=a.heads, offset=a.offset, impl=a.impl,
                                        comm=comm).to(dev, dt)
    if a.optim == "xdot":
        # one multi-tensor HIP launch per step (device-side step count when graph-captured)
        opt = xdot.FusedAdamW(model.parameters(), lr=1e-4, capturable=graph)
    else:
        opt = torch.optim.AdamW(model.parameters(), lr=1e-4, fused=(dev.type == "cuda"))
    # per-parameter buckets (the output projection's all-reduce overlaps the attention backward),
    # reduced in fp32 (one rounding to the parameter dtype at the end instead of one per ring step)
    sync = GradSync(model, comm=comm, bucket_mb=1.0, reduce_dtype=torch.float32)
    crit = xdot.MSELoss()  # fused loss + gradient pass (torch.nn.MSELoss semantics)

    g = torch.Generator(device=dev).manual_seed(1000 + rank)
    x = torch.rand(a.batch, R, a.dim, device=dev, dtype=dt, generator=g)
    y = torch.rand(a.batch, R, a.dim, device=dev, dtype=dt, generator=g)
    if a.mask == "none":
        mask = None
    elif a.mask == "zeros":
        mask = torch.zeros(a.batch, R, T, dtype=torch.bool, device=dev)
    elif a.mask == "random":
        mask = torch.rand(a.batch, R, T, device=dev, generator=g) < 0.1
        mask[..., 0] = False
    else:  # block-causal: 1024-wide blocks, each row sees its own block and every earlier one
        r = torch.arange(R, device=dev) + rank * R
        c = torch.arange(T, device=dev)
        mask = ((c[None, :] // 1024) > (r[:, None] // 1024)).unsqueeze(0).expand(a.batch, R, T).contiguous()

    def step():
        opt.zero_grad(set_to_none=True)
        out = model(x, x, x, mask)
        loss = crit(out, y)
        # == loss.backward(), minus the seed fill / scaling pass, on this thread (XDOT_INLINE_BACKWARD)
        backward(loss, unit_grad(loss))
        # with several ranks the update of the buckets already reduced runs under the last
        # gradient all-reduce (GradSync.wait(optimizer=...)); otherwise one step after the wait
        stepped = sync.wait(optimizer=None if a.no_optim or not a.split_step else opt)
        if not a.no_optim and not stepped:
            opt.step()
        return loss

    if graph:
        from xdot.utils.graphs import GraphedStep

        def body():
            out = model(x, x, x, mask)
            loss = crit(out, y)
            loss.backward()
            sync.wait()
            if not a.no_optim:
                opt.step()
            return loss

        step = GraphedStep(body, zero_grad=opt.zero_grad, warmup=max(1, warmup), optimizer=opt)
        step()  # warmup steps + capture + one replay
    else:
        for i in range(warmup):
            step()
            if dev.type == "cuda" and getattr(a, "trace", False):
                torch.cuda.synchronize()
            _trace(a, f"{dt} warmup step {i} done")
    impl = model._pick_impl(x)

    def sync_all():
        if dev.type == "cuda":
            torch.cuda.synchronize()
        comm.barrier()

    prof = None
    if profile_dir and rank == 0:
        prof = torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU,
                                                  torch.profiler.ProfilerActivity.CUDA])
        prof.__enter__()
    sync_all()
    t0 = time.perf_counter()
    for _ in range(steps):
        loss = step()
    th = time.perf_counter()  # host done enqueuing (diagnostic: close to t1 = host-bound step)
    sync_all()
    t1 = time.perf_counter()
    if prof is not None:
        prof.__exit__(None, None, None)
        os.makedirs(profile_dir, exist_ok=True)
        prof.export_chrome_trace(os.path.join(profile_dir, "trace.json"))
        with open(os.path.join(profile_dir, "ops.txt"), "w") as f:
            f.write(prof.key_averages().table(sort_by="cuda_time_total", row_limit=40))

    ms = (t1 - t0) * 1e3 / max(1, steps)
    t = torch.tensor([ms], dtype=torch.float64, device=dev if "gloo" not in comm.backend else "cpu")
    comm.all_reduce(t, op="max")
    ms = float(t.item())
    lossv = float(loss.float().item())
    if not math.isfinite(lossv):
        raise SystemExit(f"non-finite loss {lossv}")
    del model, opt, sync, x, y, mask
    return ms, (th - t0) * 1e3 / max(1, steps), lossv, impl


def _max_over_ranks(comm, dev, v: float) -> float:
    t = torch.tensor([v], dtype=torch.float64, device=dev if "gloo" not in comm.backend else "cpu")
    comm.all_reduce(t, op="max")
    return float(t.item())


def multirank_diagnostics(a, comm, dev, dt, step_ms: float, impl: str, iters: int = 10) -> dict:
    """N > 1, after the headline timing: what the step's time is made of.

    * the step's own collectives alone, at the step's sizes and chunking: the [q|v] all-gather,
      the [dq|dv] reduce-scatter (gradient wire dtype) and the per-parameter fp32 gradient
      all-reduces; ms per step and nccl-tests bus bandwidth (all-gather / reduce-scatter:
      bytes x (N-1)/N, all-reduce: x 2(N-1)/N);
    * ``compute_only_ms``: the same per-rank step with an :class:`EmulatedComm` inside each
      rank (collectives replaced by device copies of the same shapes: no transport);
    * ``exposed_comm_ms`` = step - compute-only.
    Every measurement is max over ranks; a failure becomes an ``*_error`` string, never an exit."""
    from xdot.parallel.attention import _row_chunks
    from xdot.utils.comm import EmulatedComm
    from xdot.utils.env import FLAGS

    n, rank = comm.world_size, comm.rank
    R, C, B = a.seq_len // n, a.dim, a.batch
    cuda = dev.type == "cuda"
    out = {}

    def sync():
        if cuda:
            torch.cuda.synchronize()
        comm.barrier()

    def timed(fn):
        for _ in range(3):
            fn()
        sync()
        t0 = time.perf_counter()
        for _ in range(iters):
            fn()
        sync()
        return _max_over_ranks(comm, dev, (time.perf_counter() - t0) * 1e3 / iters)

    def record(name, fn, nbytes, factor):
        try:
            ms = timed(fn)
            out[f"{name}_ms"] = round(ms, 4)
            out[f"{name}_busbw_gbps"] = round(nbytes * factor / (ms * 1e-3) / 1e9, 2)
        except Exception as e:  # noqa: BLE001
            out[f"{name}_error"] = f"{type(e).__name__}: {e}"[:300]

    chunks = _row_chunks(n, R, impl == "flash")
    gdt = torch.float32 if (FLAGS.grad_fp32 or dt == torch.float32) else dt
    try:
        xs = [torch.randn(B, rc, 2 * C, device=dev).to(dt) for _, rc in chunks]
        gbufs = [torch.empty(n, B, rc, 2 * C, device=dev, dtype=dt) for _, rc in chunks]
        parts = [torch.randn(n, B, rc, 2 * C, device=dev).to(gdt) for _, rc in chunks]
        rbufs = [torch.empty(B, rc, 2 * C, device=dev, dtype=gdt) for _, rc in chunks]
        grads = [torch.randn(C, C, device=dev) for _ in range(4)]  # the 4 weights, fp32 reduce dtype
    except Exception as e:  # noqa: BLE001
        return {"diagnostics_error": f"{type(e).__name__}: {e}"[:300]}

    def gather():
        for x, g in zip(xs, gbufs):
            comm.all_gather_into(g, x)

    def rscatter():
        for p_, r_ in zip(parts, rbufs):
            comm.reduce_scatter(r_, p_)

    def allreduce():
        hs = [comm.all_reduce(g, op="sum", async_op=True) for g in grads]
        for h in hs:
            if h is not None:
                h.wait()

    f = (n - 1) / n
    record("allgather_qv", gather, sum(g.nbytes for g in gbufs), f)
    record("reduce_scatter_dqv", rscatter, sum(p_.nbytes for p_ in parts), f)
    record("allreduce_grads", allreduce, sum(g.nbytes for g in grads), 2 * f)
    del xs, gbufs, parts, rbufs, grads
    try:
        cms = time_step(a, EmulatedComm(n, rank), dev, dt, a.steps, a.warmup)[0]
        cms = _max_over_ranks(comm, dev, cms)
        out["compute_only_ms"] = round(cms, 4)
        out["exposed_comm_ms"] = round(step_ms - cms, 4)
    except Exception as e:  # noqa: BLE001
        out["compute_only_error"] = f"{type(e).__name__}: {e}"[:300]
    return out


def _free_port() -> int:
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _child_argv(argv, gpus: int):
    """This invocation's arguments with --gpus replaced (and --sweep dropped)."""
    out, skip = [], False
    for i, x in enumerate(argv):
        if skip:
            skip = False
            continue
        if x in ("--gpus", "--sweep"):
            skip = True
            continue
        if x.startswith("--gpus=") or x.startswith("--sweep="):
            continue
        out.append(x)
    return ["--gpus", str(gpus)] + out


def _launch_cmd(argv, gpus: int):
    """Command that runs this bench as a ``gpus``-rank job: torchrun (one rank per GPU over
    RCCL, rendezvous on 127.0.0.1) for gpus > 1, a plain child for gpus == 1."""
    me = os.path.abspath(__file__)
    if gpus == 1:
        return [sys.executable, me] + _child_argv(argv, 1)
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(gpus),
            "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), me] + _child_argv(argv, gpus)


def _check_gpu_count(a) -> None:
    # torch.cuda.device_count() does not initialise HIP on this image: safe before a launch
    if a.device == "cuda" and a.backend != "gloo":  # gloo rehearsals may share one GPU
        have = torch.cuda.device_count()
        if have and a.gpus > have:
            print(f"bench.py: --gpus {a.gpus} but only {have} GPU(s) visible", file=sys.stderr, flush=True)
            raise SystemExit(2)


def self_launch(argv, a) -> int:
    """``python bench.py --gpus N`` without a launcher (no WORLD_SIZE in the environment):
    start the N-rank job ourselves, BEFORE any GPU call in this process, as a torchrun child
    (the reference's equivalent is ``horovodrun -np N``, README.md:77).  The child's rank 0
    prints the one JSON line on our stdout; its exit code is ours."""
    import subprocess

    _check_gpu_count(a)
    return subprocess.call(_launch_cmd(argv, a.gpus))


def sweep(argv, ns) -> int:
    """``--sweep 1,2,4,8``: each N in fresh processes, one JSON line per N (rank 0's record),
    then one summary line with the speed-up and strong-scaling efficiency against the N=1 run."""
    import subprocess

    recs = {}
    rc_all = 0
    for n in ns:
        p = subprocess.run(_launch_cmd(argv, n), stdout=subprocess.PIPE, text=True)
        lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
        if p.returncode != 0 or not lines:
            print(json.dumps({"sweep_n": n, "error": f"exit {p.returncode}"}), flush=True)
            rc_all = rc_all or (p.returncode or 1)
            continue
        rec = json.loads(lines[-1])
        recs[n] = rec
        print(json.dumps(rec), flush=True)
    if recs:
        base_n = min(recs)
        base = recs[base_n]["ms_per_step"] * base_n
        summ = {"sweep": sorted(recs), "ms_per_step": {n: recs[n]["ms_per_step"] for n in sorted(recs)},
                "speedup_vs_n1": {n: round(recs[base_n]["ms_per_step"] / recs[n]["ms_per_step"], 3) for n in sorted(recs)}
                if base_n == 1 else None,
                "strong_scaling_efficiency": {n: round(base / (n * recs[n]["ms_per_step"]), 3) for n in sorted(recs)},
                "metric": recs[base_n]["metric"]}
        print(json.dumps(summ), flush=True)
    return rc_all


def main(argv=None, comm=None):
    """``comm``: optional communicator override (``benchmarks/bench_rank.py`` passes an
    :class:`xdot.utils.comm.EmulatedComm` to run one rank of an N-GPU step on one GPU)."""
    raw = list(sys.argv[1:] if argv is None else argv)
    a = parse(argv)
    if comm is None and a.sweep:
        raise SystemExit(sweep(raw, [int(x) for x in a.sweep.split(",") if x.strip()]))
    if comm is None and a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        raise SystemExit(self_launch(raw, a))
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from xdot.utils import comm as C
    from xdot.utils.env import FLAGS

    emulated = comm is not None
    comm = comm or C.init(a.backend)
    n, rank = comm.world_size, comm.rank
    if n != a.gpus and not emulated:
        # the job must be the N-rank job it claims to be (reference: utils/comm.py:8-9 asserts
        # hvd.size() == the MPI world size at init)
        msg = f"bench.py: --gpus {a.gpus} but the launch has {n} rank(s); start it with torchrun --nproc-per-node {a.gpus}"
        print(msg, file=sys.stderr, flush=True)
        raise SystemExit(2)
    dev = torch.device(a.device, C.get_local_rank() % max(1, torch.cuda.device_count())) if a.device == "cuda" \
        else torch.device("cpu")
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
    dt = {"bf16": torch.bfloat16, "fp16": torch.float16, "fp32": torch.float32}[a.dtype]
    T = a.seq_len
    if T % n:
        raise SystemExit(f"seq-len {T} not divisible by world size {n}")
    R = T // n

    check_err = None
    _trace(a, "init done")
    if not emulated and not a.no_check:
        check_err = numerics_check(a, comm, dev, dt, a.impl)
    _trace(a, "numerics check done")
    ms, host_ms, lossv, impl = time_step(a, comm, dev, dt, a.steps, a.warmup, graph=a.graph,
                                         profile_dir=a.profile_dir)
    diag = {}
    if n > 1 and not emulated and a.diagnostics:
        _trace(a, "multi-rank diagnostics start")
        diag = multirank_diagnostics(a, comm, dev, dt, ms, impl)
        _trace(a, "multi-rank diagnostics done")
    fp32 = {}
    if a.fp32_steps > 0 and dt != torch.float32 and dev.type == "cuda":
        # the reference computes in fp32 only (module.py:60-71): time the same step in fp32 too,
        # under both fp32 kernel families (XDOT_FP32_MODE: exact fp32 MFMA default, split-bf16)
        default_mode = FLAGS.fp32_mode
        try:
            for mode in [default_mode] + [m for m in ("split", "exact") if m != default_mode]:
                FLAGS.fp32_mode = mode
                _trace(a, f"fp32 {mode} start")
                fp32[mode] = time_step(a, comm, dev, torch.float32, a.fp32_steps, a.fp32_warmup)
                _trace(a, f"fp32 {mode} done: {fp32[mode][0]:.2f} ms")
        finally:
            FLAGS.fp32_mode = default_mode
    if rank == 0 or emulated:  # an emulated rank is the only process: it reports
        metric = METRIC
        if (T, a.dim, a.heads) != (25000, 768, 8):  # not the headline config: say what was run
            metric = f"ms/fwd+bwd DistributedDotProductAttn T={T} d={a.dim} h={a.heads}"
        from xdot.parallel.attention import _row_chunks

        backend = comm.backend
        transport = {"nccl": "rccl", "ipc+nccl": "ipc+rccl"}.get(backend, backend)
        rccl = None
        if "nccl" in backend:
            try:
                rccl = ".".join(map(str, torch.cuda.nccl.version()))
            except Exception:  # noqa: BLE001
                rccl = "unknown"
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
            "host_enqueue_ms_per_step": round(host_ms, 4),
            "loss": lossv,
            "world_size": n,
            "rank": rank,
            "transport": transport,
            "rccl_version": rccl,
            "gather_chunks": len(_row_chunks(n, R, impl == "flash")),
            "local_first": bool(FLAGS.local_first),
            "numerics_check_max_rel_err": None if check_err is None else round(check_err, 5),
        }
        rec.update(diag)
        if fp32:
            first = next(iter(fp32))
            rec["fp32_ms_per_step"] = round(fp32[first][0], 4)
            rec["fp32_impl"] = f"{fp32[first][3]}/{first}"
            for mode, r in fp32.items():
                rec[f"fp32_{mode}_ms_per_step"] = round(r[0], 4)
            rec["fp32_steps"] = a.fp32_steps
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
