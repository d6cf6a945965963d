#!/bin/bash
# Occupancy (waves/SIMD) and column-split sweep of the flash kernels at the N=1 and N=8 headline shapes.
set -e
O=gpurun_out/exp
mkdir -p $O
for w in 2 1; do
  XDOT_FA_WPS=$w timeout -k 10 120 python benchmarks/bench_flash.py --mask --iters 10 > $O/wps${w}_n1.log 2>&1
  XDOT_FA_WPS=$w timeout -k 10 120 python benchmarks/bench_flash.py --mask --iters 20 --R 3125 > $O/wps${w}_n8.log 2>&1
  for s in 1 2 3 4 5 6; do
    XDOT_FA_WPS=$w timeout -k 10 120 python benchmarks/bench_flash.py --mask --iters 10 --nsplit $s --only fwd >> $O/split_w${w}.log 2>&1
    XDOT_FA_WPS=$w timeout -k 10 120 python benchmarks/bench_flash.py --mask --iters 10 --nsplit $s --only bwd_rows >> $O/split_w${w}.log 2>&1
  done
done
echo done
