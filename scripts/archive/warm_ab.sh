#!/bin/bash
# bench.py default K/W (10 / 3) vs a longer warmup (20 / 10), interleaved on one box.
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/warm_ab.log
for a in "" "--warmup 10 --steps 20" "" "--warmup 10 --steps 20"; do
  timeout -k 10 200 python bench.py $a --fp32-steps 0 --no-check > gpurun_out/warm_one.json 2>/dev/null || exit 1
  python -c "import json;r=json.loads([l for l in open('gpurun_out/warm_one.json') if 'metric' in l][-1]);print('[$a]', r['ms_per_step'])" >> gpurun_out/warm_ab.log || exit 1
done
cat gpurun_out/warm_ab.log
