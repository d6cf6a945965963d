"""HIP-graph replay vs eager, with the fused backward on the default stream rule (None), forced
two streams (False) or forced one stream (True) (``xdot.parallel.attention.ONE_STREAM_BACKWARD``),
at N=1 and emulated per-rank shapes.
Prints bench.py's JSON lines tagged with the variant.

    python benchmarks/graph_ab.py --world 1 8 --steps 10 --warmup 3
"""
import argparse
import io
import json
import os
import sys
from contextlib import redirect_stdout

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, nargs="+", default=[1, 8])
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    a = ap.parse_args()
    import bench
    import xdot.parallel.attention as A
    from xdot.utils.comm import EmulatedComm

    for n in a.world:
        for one in (None, False, True):
            for graph in (False, True):
                A.ONE_STREAM_BACKWARD = one
                args = ["--gpus", str(n), "--steps", str(a.steps), "--warmup", str(a.warmup), "--fp32-steps", "0",
                        "--no-check"] + (["--graph"] if graph else [])
                buf = io.StringIO()
                with redirect_stdout(buf):
                    bench.main(args, comm=EmulatedComm(n) if n > 1 else None)
                for line in buf.getvalue().splitlines():
                    if line.startswith("{"):
                        r = json.loads(line)
                        print(json.dumps({"world": n, "one_stream_bwd": one, "graph": graph, "ms": r["value"],
                                          "host_ms": r["host_enqueue_ms_per_step"]}), flush=True)


if __name__ == "__main__":
    main()
