#!/bin/bash
# Quick regression check of the step: N=1 and emulated N=8, default vs --no-split-step, 2 rounds.
set -o pipefail
O=gpurun_out/${1:-regress}
mkdir -p $O
for r in 1 2; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 >> $O/n1.log 2>&1 || exit $?
  timeout -k 10 200 python benchmarks/bench_rank.py --world 8 --steps 20 --warmup 5 >> $O/n8.log 2>&1 || exit $?
  timeout -k 10 200 python benchmarks/bench_rank.py --world 8 --steps 20 --warmup 5 --no-split-step >> $O/n8_nosplit.log 2>&1 || exit $?
done
echo regress-ok
