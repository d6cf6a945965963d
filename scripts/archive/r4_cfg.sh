#!/bin/bash
# Round-end BASELINE config re-measure at HEAD: masked steps (random 10 % / block-causal vs
# all-False, interleaved), long context T=200000 (N=1 and one rank of 8), emulated N=2/4 ranks.
set -o pipefail
T=${1:-r4cfg}
O=gpurun_out/$T; mkdir -p $O
for r in 1 2; do
  for m in zeros random block-causal; do
    timeout -k 10 200 python bench.py --mask $m --steps 20 --warmup 5 --fp32-steps 0 --no-check 2>&1 | grep '"metric"' | sed "s/^/$m /" >> $O/mask.log || exit $?
  done
done
timeout -k 10 300 python benchmarks/bench_rank.py --world 8 --seq-len 200000 --steps 3 --warmup 1 > $O/c5_n8.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --seq-len 200000 --steps 2 --warmup 1 --fp32-steps 0 --no-check > $O/c5_n1.log 2>&1 || exit $?
for w in 2 4; do
  timeout -k 10 200 python benchmarks/bench_rank.py --world $w --steps 20 --warmup 5 --fp32-steps 0 > $O/r$w.log 2>&1 || exit $?
done
echo cfg-ok
