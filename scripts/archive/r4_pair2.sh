#!/bin/bash
# Paired weight-gradient launch vs two launches, interleaved on one box.
set -o pipefail
T=${1:-r4pair2}
O=gpurun_out/$T
mkdir -p $O
for rep in 1 2 3; do
  for p in 1 0; do
    XDOT_WGRAD_PAIR=$p timeout -k 10 200 python bench.py --steps 20 --warmup 5 --fp32-steps 0 --no-check > $O/n1_p${p}_$rep.log 2>&1 || exit $?
    XDOT_WGRAD_PAIR=$p timeout -k 10 200 python benchmarks/bench_rank.py --world 8 --steps 30 --warmup 5 --fp32-steps 0 > $O/r8_p${p}_$rep.log 2>&1 || exit $?
  done
done
echo pair2-ok
