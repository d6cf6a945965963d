"""Markdown table: the reference's benchmark_results/*.json (median distributed_time, cold and
unsynced) vs xdot's same-schema records (cold unsynced replica and synced p50).

    python scripts/ref_table.py /root/reference/benchmark_results benchmark_results
"""
import glob
import json
import os
import statistics
import sys

ref_dir, ours_dir = sys.argv[1], sys.argv[2]
print("| file | reference median distributed_time s, cold, unsynced (records) | xdot cold unsynced s | "
      "xdot synced median s (records) | speed-up (ref median / xdot median) |")
print("|---|---|---|---|---|")
for f in sorted(glob.glob(os.path.join(ours_dir, "*.json"))):
    name = os.path.basename(f)
    rp = os.path.join(ref_dir, name)
    if not os.path.exists(rp):
        continue
    ref = json.load(open(rp))  # plain JSON (safe loader)
    recs = json.load(open(f))
    ours = [r for r in recs if "cold_unsynced_s" in r][-1]  # the summary record (trial records follow it)
    trials = [r["distributed_time"] for r in recs if "trial" in r]
    rm = statistics.median(r["distributed_time"] for r in ref)
    p50 = statistics.median(trials) if trials else ours["ms_p50"] / 1e3
    print(f"| `{name}` | {rm:.4f} ({len(ref)}) | {ours['cold_unsynced_s']:.4f} | {p50:.5f} ({len(trials) or 1}) "
          f"| {rm / p50:.0f}x |")
