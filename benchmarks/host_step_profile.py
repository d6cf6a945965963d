"""Host-side (Python) cost of the timed steps only: cProfile around bench.time_step's loop at the
emulated N-rank shape (EmulatedComm: no transport), top functions by own time.

    python benchmarks/host_step_profile.py --world 8 --steps 40
"""
import argparse
import cProfile
import io
import os
import pstats
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--inline-backward", action="store_true",
                    help="run backward on the calling thread (torch.autograd.set_multithreading_enabled(False)) "
                         "so cProfile sees the Python backward functions too")
    a = ap.parse_args()
    import torch

    import bench
    from xdot.utils.comm import EmulatedComm

    args = bench.parse(["--gpus", str(a.world), "--fp32-steps", "0", "--no-check"])
    comm = EmulatedComm(a.world)
    dev = torch.device("cuda", 0)
    bench.time_step(args, comm, dev, torch.bfloat16, 5, 5)  # warm everything (kernels, caches, allocator)
    ms0, host0, _, _ = bench.time_step(args, comm, dev, torch.bfloat16, a.steps, 2)
    print(f"world {a.world}: {ms0:.3f} ms/step, host enqueue {host0:.3f} ms/step (unprofiled, engine thread)")
    if a.inline_backward:
        torch.autograd.set_multithreading_enabled(False)
        bench.time_step(args, comm, dev, torch.bfloat16, 5, 5)
        ms0, host0, _, _ = bench.time_step(args, comm, dev, torch.bfloat16, a.steps, 2)
        print(f"world {a.world}: {ms0:.3f} ms/step, host enqueue {host0:.3f} ms/step (unprofiled, inline backward)")
    pr = cProfile.Profile()
    pr.enable()
    ms, host_ms, _, _ = bench.time_step(args, comm, dev, torch.bfloat16, a.steps, 2)
    pr.disable()
    print(f"world {a.world}: {ms:.3f} ms/step, host enqueue {host_ms:.3f} ms/step (profiled)")
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(a.top)
    print(s.getvalue())
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("cumulative").print_stats(a.top)
    print(s.getvalue())


if __name__ == "__main__":
    main()
