#!/bin/bash
# same-box A/B of gemm3 builds: VARIANTS="name:ext_path:env ..." alternated for 2 rounds
set -e
O=gpurun_out/gemm3_ab
mkdir -p $O
C=${CASES:-nt,nt_small,nt_rank8,ntk3072,all}
for r in 1 2; do
  for v in $VARIANTS; do
    name=${v%%:*}; rest=${v#*:}; ext=${rest%%:*}; envs=${rest#*:}
    echo "== round $r variant $name" >> $O/ab.log
    env XDOT_EXT_PATH=$ext $envs timeout -k 10 300 python -u benchmarks/bench_gemm.py --path v3 --cases $C --iters 10 >> $O/ab.log 2>&1
  done
done
python - <<'PY'
import json, collections
res = collections.defaultdict(list); cur = None
for line in open("gpurun_out/gemm3_ab/ab.log"):
    if line.startswith("=="): cur = line.split()[-1]; continue
    if line.startswith("{"):
        d = json.loads(line); res[(d["case"], cur)].append((d["xdot_ms"], d["torch_ms"]))
for k in sorted(res): print(k, res[k])
PY
