"""Per-step GPU timeline from a rocprofv3 kernel trace (rocpd ``*.db`` or ``*kernel_trace.csv``).

Splits the trace into steps at a marker kernel (default: the fused AdamW kernel that ends every
``bench.py`` step) and reports, for the last complete step, each kernel's start offset,
duration and the idle gap before it, plus busy/idle totals averaged over the last N steps.

    python scripts/step_timeline.py gpurun_out/rank8/run_results.db --steps 10
"""
from __future__ import annotations

import argparse
import csv
import sqlite3


def load(path):
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        rows = c.execute("select name, start, end from kernels order by start").fetchall()
        return [(n, int(s), int(e)) for n, s, e in rows]
    with open(path) as f:
        r = csv.DictReader(f)
        rows = [(d["Kernel_Name"], int(d["Start_Timestamp"]), int(d["End_Timestamp"])) for d in r]
    return sorted(rows, key=lambda x: x[1])


def short(n, w=60):
    n = n.split("(")[0]
    return n if len(n) <= w else n[: w - 3] + "..."


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--marker", default="adam", help="substring (case-insensitive) of the last kernel of a step")
    a = ap.parse_args()
    ks = load(a.trace)
    ends = [i for i, k in enumerate(ks) if a.marker in k[0].lower()]
    # a step may launch several marker kernels back to back: keep the last of each run
    ends = [i for j, i in enumerate(ends) if j + 1 == len(ends) or ends[j + 1] != i + 1]
    if len(ends) < 2:
        raise SystemExit("fewer than 2 steps found")
    steps = list(zip(ends[:-1], ends[1:]))[-a.steps:]
    tot_span = tot_busy = 0
    for s, e in steps:
        seg = ks[s + 1: e + 1]
        span = seg[-1][2] - ks[s][2]
        busy = sum(k[2] - k[1] for k in seg)
        tot_span += span
        tot_busy += busy
    n = len(steps)
    print(f"steps={n}  span/step={tot_span / n / 1e6:.3f} ms  kernel-busy/step={tot_busy / n / 1e6:.3f} ms  "
          f"idle/step={(tot_span - tot_busy) / n / 1e6:.3f} ms  kernels/step={steps[-1][1] - steps[-1][0]}")
    s, e = steps[-1]
    t0 = ks[s][2]
    prev = t0
    print(f"{'start_us':>9} {'dur_us':>8} {'gap_us':>7}  kernel")
    for k in ks[s + 1: e + 1]:
        print(f"{(k[1] - t0) / 1e3:9.1f} {(k[2] - k[1]) / 1e3:8.1f} {(k[1] - prev) / 1e3:7.1f}  {short(k[0])}")
        prev = max(prev, k[2])


if __name__ == "__main__":
    main()
