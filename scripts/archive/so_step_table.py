"""Summarise scripts/archive/so_step_ab2.sh: per variant, kernel medians (bench_flash) and step medians."""
import collections
import json
import os
import statistics
import sys

d = sys.argv[1]
for v in sys.argv[2:]:
    rows = collections.defaultdict(list)
    for name in (f"{v}.log", f"step_{v}.log"):
        path = os.path.join(d, name)
        if not os.path.exists(path):
            continue
        for line in open(path):
            if not line.startswith("{"):
                continue
            r = json.loads(line)
            if "kernel" in r:
                rows[f"{r['kernel']}@R{r.get('R')}"].append(r["ms"])
            else:
                rows[f"step N={r['n_gpus']}{' emu' if 'EMULATED' in r['metric'] else ''}"].append(r["value"])
    print(v, " | ".join(f"{k} {statistics.median(x):.4f} ({' '.join(f'{y:.3f}' for y in x)})" for k, x in rows.items()))
