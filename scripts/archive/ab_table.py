"""Summarise scripts/archive/ab.sh logs: per kernel, min and median of the per-run medians."""
import collections
import json
import statistics
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/ab"
vs = sys.argv[2].split(",") if len(sys.argv) > 2 else ["A", "B"]
for v in vs:
    ms = collections.defaultdict(list)
    for line in open(f"{d}/{v}.log"):
        if line.startswith("{"):
            r = json.loads(line)
            ms[r["kernel"] + ("@R" + str(r.get("R")))].append(r["ms"])
    print(v, "  ".join(f"{k}: min {min(x):.4f} med {statistics.median(x):.4f}" for k, x in ms.items()))
