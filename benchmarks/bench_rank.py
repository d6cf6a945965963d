"""One rank of an N-GPU headline step, emulated on ONE GPU (diagnostics, not the headline).

Runs ``bench.py``'s exact training step with an :class:`xdot.utils.comm.EmulatedComm`: the
rank owns T/N rows and gathers/reduce-scatters full-size buffers, but the collectives are
device-local copies.  The result is the per-rank compute + launch cost of the N-GPU step
(what the scaling run adds on top is the RCCL transport).  Prints ``bench.py``'s JSON line
with the metric and parallelism marked EMULATED.

    python benchmarks/bench_rank.py --world 8 --steps 20 --warmup 5
"""
from __future__ import annotations

import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--world", type=int, nargs="+", default=[8])
    a, rest = ap.parse_known_args()
    import bench
    from xdot.utils.comm import EmulatedComm

    for n in a.world:
        bench.main(["--gpus", str(n)] + rest, comm=EmulatedComm(n))


if __name__ == "__main__":
    main()
