"""Summarise scripts/archive/so_ab.sh: per variant, kernel medians (bench_flash) per shape."""
import collections
import json
import statistics
import sys

d = sys.argv[1]
for v in sys.argv[2:]:
    ks = collections.defaultdict(list)
    for line in open(f"{d}/{v}.log"):
        if line.startswith("{"):
            r = json.loads(line)
            ks[f"{r['kernel']}@R{r.get('R')}"].append(r["ms"])
    print(v, " | ".join(f"{k} {statistics.median(x):.4f} ({' '.join(f'{y:.3f}' for y in x)})" for k, x in ks.items()))
