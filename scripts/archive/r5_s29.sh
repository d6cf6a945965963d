#!/bin/bash
# Round 5 pass 29: upper bound of a cheaper staging for the exact-fp32 kernels -- timing-only build
# with no tile staging at all (XDOT_AB_NOSTAGE: wrong results) vs HEAD, interleaved
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r5s29; mkdir -p $OUT
for rep in 1 2; do
  for v in "" _nostage; do
    XDOT_EXT_PATH=$GRAFT_REPO_ROOT/xdot/_C$v.so timeout -k 10 200 python benchmarks/bench_flash.py --dtype fp32 --fp32-mode exact --iters 5 --scores > $OUT/exact$v.$rep.log 2>&1 || exit $?
  done
done
