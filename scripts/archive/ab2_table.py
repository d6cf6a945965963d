"""Summarise scripts/archive/env_ab2.sh: per arm, kernel medians (bench_flash) and step medians."""
import collections
import json
import statistics
import sys

d = sys.argv[1]
for tag in ("A", "B"):
    ks = collections.defaultdict(list)
    for line in open(f"{d}/{tag}.log"):
        if line.startswith("{"):
            r = json.loads(line)
            ks[f"{r['kernel']}@R{r.get('R')}"].append(r["ms"])
    st = collections.defaultdict(list)
    for line in open(f"{d}/step_{tag}.log"):
        if line.startswith("{"):
            r = json.loads(line)
            st[f"step N={r['n_gpus']}{' emu' if 'EMULATED' in r['metric'] else ''}"].append(r["value"])
    print(tag, " | ".join(f"{k} {statistics.median(v):.4f} ({' '.join(f'{x:.3f}' for x in v)})"
                         for k, v in list(ks.items()) + list(st.items())))
