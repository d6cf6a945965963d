"""Median table of an alternating bench_rank A/B log (scripts/archive/gpu_overlap_ab.sh)."""
import json
import statistics
import sys
from collections import defaultdict

res = defaultdict(list)
cfg = None
for line in open(sys.argv[1]):
    if line.startswith("=="):
        cfg = " ".join(w for w in line[2:].split() if not w.startswith("round="))
    elif line.startswith("{"):
        r = json.loads(line)
        res[(cfg, r["n_gpus"])].append(r["value"])
for (cfg, n), v in sorted(res.items(), key=lambda kv: (kv[0][1], kv[0][0])):
    print(f"| N={n} | {cfg} | {statistics.median(v):.3f} | {' '.join(f'{x:.3f}' for x in v)} |")
