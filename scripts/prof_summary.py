"""Condense a rocprofv3 ``*_kernel_stats.csv`` into a short markdown table.

    python scripts/prof_summary.py gpurun_out/prof_flash/prof_kernel_stats.csv --steps 4 > profiles/x.md

``--steps`` divides totals by the number of profiled steps (warmup + timed) to give
per-step milliseconds.
"""
import argparse
import csv
import re


def short(name: str) -> str:
    name = re.sub(r"\(.*", "", name)
    if name.startswith("Cijk_"):
        return "hipBLASLt " + name.split("_MT")[1].split("_")[0] if "_MT" in name else "hipBLASLt"
    name = name.replace("void ", "")
    if "at::native::" in name:
        m = re.search(r"at::native::(?:\(anonymous namespace\)::)?([A-Za-z_]+)", name)
        return "aten " + (m.group(1) if m else name[:40])
    return name[:90]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--steps", type=float, default=1.0)
    ap.add_argument("--top", type=int, default=15)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.csv)))
    total = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"| kernel | calls | ms/step | avg us | % |\n|---|---|---|---|---|")
    for r in rows[: a.top]:
        t = float(r["TotalDurationNs"])
        print(f"| `{short(r['Name'])}` | {r['Calls']} | {t / 1e6 / a.steps:.3f} | "
              f"{float(r['AverageNs']) / 1e3:.1f} | {100 * t / total:.1f} |")
    print(f"\nGPU kernel time per step: {total / 1e6 / a.steps:.3f} ms")


if __name__ == "__main__":
    main()
