#!/bin/bash
# Round 5 pass 22: fp32 kernels with and without the score buffer at HEAD (row splits, fp32
# split model) -- sizing a dS-only buffer mode for the split family
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r5s22; mkdir -p $OUT
export XDOT_EXT_PATH=$GRAFT_REPO_ROOT/xdot/_C.so
for m in split exact; do
  timeout -k 10 200 python benchmarks/bench_flash.py --dtype fp32 --fp32-mode $m --iters 5 > $OUT/${m}_recompute.log 2>&1 || exit $?
  timeout -k 10 200 python benchmarks/bench_flash.py --dtype fp32 --fp32-mode $m --iters 5 --scores > $OUT/${m}_scores.log 2>&1 || exit $?
done
