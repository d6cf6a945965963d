#!/bin/bash
set -o pipefail
O=gpurun_out/r2_qsweep
mkdir -p $O
for T in 24576 25000 26112 28672 32768; do
  timeout -k 10 120 python benchmarks/bench_flash.py --R 3125 --T $T --iters 10 --concurrent >> $O/sweep.log 2>&1 || exit $?
done
echo q-ok
