#!/bin/bash
# Round 5 pass 35: emulated N = 8 rank step vs the row kernel's column splits (XDOT_ROWS_SPLIT)
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r5s35; mkdir -p $OUT
export XDOT_EXT_PATH=$GRAFT_REPO_ROOT/xdot/_C.so
for rep in 1 2; do
  for rs in 0 2 3 4 8 12; do
    XDOT_ROWS_SPLIT=$rs timeout -k 10 300 python benchmarks/bench_rank.py --world 8 > $OUT/rs$rs.$rep.log 2>&1 || exit $?
  done
done
