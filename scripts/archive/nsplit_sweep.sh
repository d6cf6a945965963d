#!/bin/bash
# Column-split sweep of the flash forward / backward-rows kernels at the N=1 and N=8 per-rank
# shapes (benchmarks/bench_flash.py --nsplit; 0 = the pick_split heuristic).
O=gpurun_out/nsplit
mkdir -p $O
rm -f $O/*.log
for R in 25000 3125; do
  for s in 0 1 2 3 4 5 6; do
    timeout -k 10 120 python benchmarks/bench_flash.py --R $R --mask --nsplit $s --iters 20 > $O/r${R}_s$s.log 2>&1 || exit 1
    echo "R=$R nsplit=$s $(grep -o '"kernel": "[a-z_]*", "ms": [0-9.]*' $O/r${R}_s$s.log | sed 's/"kernel": //; s/, "ms"//' | tr '\n' ' ')"
  done
done
