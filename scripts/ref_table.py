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
print("| file | reference median distributed_time s (cold, unsynced) | xdot cold unsynced s | xdot synced p50 s | speed-up (ref median / xdot p50) |")
print("|---|---|---|---|---|")
for f in sorted(glob.glob(os.path.join(ours_dir, "*.json"))):
    name = os.path.basename(f)
    rp = os.path.join(ref_dir, name)
    if not os.path.exists(rp):
        continue
    ref = json.load(open(rp))  # plain JSON (safe loader)
    ours = json.load(open(f))[-1]
    rm = statistics.median(r["distributed_time"] for r in ref)
    p50 = ours["ms_p50"] / 1e3
    print(f"| `{name}` | {rm:.4f} | {ours['cold_unsynced_s']:.4f} | {p50:.5f} | {rm / p50:.0f}x |")
