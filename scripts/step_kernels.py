"""Per-step kernel table from a rocprofv3 kernel trace of bench.py / bench_rank.py: the window
between the first and the last AdamW launch (one optimizer launch per parameter group per step).

    python scripts/step_kernels.py gpurun_out/profstep/prof/prof_kernel_trace.csv [--top 16]

Prints steps in the window, ms/step from the timestamps, and per kernel: calls/step, µs/step and
average µs (concurrent kernels overlap, so µs/step sums can exceed the step).
"""
import argparse
import collections
import csv
import re


def short(n: str) -> str:
    n = re.sub(r"\(.*", "", n).replace("void ", "")
    if n.startswith("Cijk_") and "_MT" in n:
        return "hipBLASLt " + n.split("_MT")[1].split("_")[0]
    return n[:72]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--top", type=int, default=16)
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    ad = [i for i, r in enumerate(rows) if "adamw_kernel" in r["Kernel_Name"]]
    # one mse_final per step: steps = number of mse_final launches after the first AdamW
    mse = [i for i, r in enumerate(rows) if "mse_final" in r["Kernel_Name"] and i > ad[0]]
    steps = len(mse)
    lo, hi = ad[0], ad[-1]
    agg = collections.defaultdict(lambda: [0, 0.0])
    for r in rows[lo + 1:hi + 1]:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        e = agg[short(r["Kernel_Name"])]
        e[0] += 1
        e[1] += d
    span = (int(rows[hi]["End_Timestamp"]) - int(rows[lo]["End_Timestamp"])) / 1e6
    print(f"{steps} steps in the window, {span / steps:.3f} ms/step (timestamps)\n")
    print("| kernel | calls/step | µs/step | avg µs |\n|---|---|---|---|")
    for k, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:a.top]:
        print(f"| `{k}` | {c / steps:.1f} | {t / steps:.1f} | {t / c:.1f} |")


if __name__ == "__main__":
    main()
