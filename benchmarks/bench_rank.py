"""One rank of an N-GPU headline step, emulated on ONE GPU (diagnostics, not the headline).

Runs ``bench.py``'s exact training step with an :class:`xdot.utils.comm.EmulatedComm`: the
rank owns T/N rows and gathers/reduce-scatters full-size buffers, but the collectives are
device-local copies.  The result is the per-rank compute + launch cost of the N-GPU step
(what the scaling run adds on top is the RCCL transport).  Prints ``bench.py``'s JSON line
with the metric and parallelism marked EMULATED.

``--link-gbps G`` turns on the link model: every collective runs on its own stream as a
spin of (bytes on the wire / G GB/s) plus the copy, so the step shows how much of an
xGMI-sized transfer the schedule hides (an ASSUMED rate, not a measurement of RCCL).

    python benchmarks/bench_rank.py --world 8 --steps 20 --warmup 5
    python benchmarks/bench_rank.py --world 8 --link-gbps 300 --p2p-gbps 64
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
    ap.add_argument("--link-gbps", type=float, default=None,
                    help="emulated collective bus bandwidth per rank (GB/s); default: no transfer time")
    ap.add_argument("--p2p-gbps", type=float, default=None, help="emulated ring-hop link rate (GB/s)")
    ap.add_argument("--rank", type=int, default=0,
                    help="which rank to emulate (the segmented forward launches one partial per peer range: "
                         "a middle rank has two ranges per gather chunk, rank 0 one)")
    ap.add_argument("--no-seg-merge", action="store_true",
                    help="(A/B) a middle rank runs one forward partial per peer range instead of one per chunk")
    a, rest = ap.parse_known_args()
    if a.no_seg_merge:
        import xdot.parallel.attention as pa

        pa.SEGMENT_MERGE = False
    import bench
    from xdot.utils.comm import EmulatedComm

    for n in a.world:
        bench.main(["--gpus", str(n)] + rest, comm=EmulatedComm(n, rank=min(a.rank, n - 1), link_gbps=a.link_gbps,
                                                                  p2p_gbps=a.p2p_gbps))


if __name__ == "__main__":
    main()
