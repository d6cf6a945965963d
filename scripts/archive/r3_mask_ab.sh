#!/bin/bash
# Masked vs unmasked headline step on ONE box, interleaved (zeros, random, zeros, random,
# block-causal): the ratio is taken within the run (box-to-box spread is 5-7 %).
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/mask_ab.log
: > $L
for m in zeros random zeros random block-causal; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --fp32-steps 0 --no-check --mask $m > gpurun_out/mask_$m.json 2>> $L || exit 1
  python -c "import json,sys;r=json.loads(open('gpurun_out/mask_$m.json').read().strip().splitlines()[-1]);print('$m', r['ms_per_step'])" >> $L || exit 1
done
cat $L | grep -v Warning
