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
    ap.add_argument("--seq-len", type=int, default=25000)
    ap.add_argument("--one-stream", action="store_true",
                    help="(A/B) one-stream attention backward (xdot.parallel.attention.ONE_STREAM_BACKWARD)")
    ap.add_argument("--inline-backward", action="store_true",
                    help="(default now: XDOT_INLINE_BACKWARD=1) kept for old scripts")
    a = ap.parse_args()
    import torch

    import bench
    from xdot.utils.comm import EmulatedComm
    from xdot.utils.env import FLAGS

    args = bench.parse(["--gpus", str(a.world), "--seq-len", str(a.seq_len), "--fp32-steps", "0", "--no-check"])
    comm = EmulatedComm(a.world) if a.world > 1 else None
    if comm is None:
        from xdot.utils.comm import LocalComm

        comm = LocalComm()
    if a.one_stream:
        import xdot.parallel.attention as pa

        pa.ONE_STREAM_BACKWARD = True
    dev = torch.device("cuda", 0)
    inline = FLAGS.inline_backward
    bench.time_step(args, comm, dev, torch.bfloat16, 5, 5)  # warm everything (kernels, caches, allocator)
    for mode in (False, True):  # autograd's device worker thread, then the calling thread
        FLAGS.inline_backward = mode
        ms0, host0, _, _ = bench.time_step(args, comm, dev, torch.bfloat16, a.steps, 2)
        print(f"world {a.world}: {ms0:.3f} ms/step, host enqueue {host0:.3f} ms/step "
              f"(unprofiled, {'inline backward' if mode else 'engine thread'})")
    FLAGS.inline_backward = inline
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
