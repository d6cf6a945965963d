"""Probe: does HIP stream capture keep a side stream's priority on its kernel nodes, and can the
priority attribute of a captured kernel node be set?  A captured two-stream backward needs one
of the two to replay its gathered-side branch at high priority (profiles/r3_graph.md).

    python benchmarks/micro/graph_prio_probe.py

ROCm 7.2 / torch 2.10 on MI355X: capture records priority 0 on every node, and
hipGraphKernelNodeSetAttribute(.., hipKernelNodeAttributePriority, ..) returns invalid argument.
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import xdot  # noqa: E402,F401  (loads the extension)
from xdot import _ext  # noqa: E402


def main():
    ops = _ext.ops()
    a = torch.randn(1024, 1024, device="cuda")
    hi = torch.cuda.Stream(priority=-1)
    print("stream priorities: cur", torch.cuda.current_stream().priority, "hi", hi.priority, flush=True)
    g = torch.cuda.CUDAGraph(keep_graph=True)
    with torch.cuda.graph(g):
        b = a * 2
        hi.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(hi):
            c = a + 1
        torch.cuda.current_stream().wait_stream(hi)
        d = b + c
    raw = g.raw_cuda_graph()
    print("kernel node priorities after capture:", list(ops.graph_kernel_priorities(raw)), flush=True)
    try:
        ops.graph_set_kernel_priority(raw, 1, int(hi.priority))
        print("set node 1 priority", hi.priority, "->", list(ops.graph_kernel_priorities(raw)), flush=True)
    except Exception as e:  # noqa: BLE001
        print("set node 1 priority", hi.priority, "failed:", e, flush=True)
    torch.cuda.synchronize()  # a failed HIP call leaves its error for the next one: consume it here
    d.zero_()
    g.replay()
    torch.cuda.synchronize()
    print("replay max err:", float((d - (a * 2 + (a + 1))).abs().max()), flush=True)


if __name__ == "__main__":
    main()
