#!/bin/bash
# Round 5 pass 33: bf16 N=1 step vs the row kernel's column splits (XDOT_ROWS_SPLIT; 0 = auto)
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r5s33; mkdir -p $OUT
export XDOT_EXT_PATH=$GRAFT_REPO_ROOT/xdot/_C.so
for rep in 1 2; do
  for rs in 0 1 2 4 6 8; do
    XDOT_ROWS_SPLIT=$rs timeout -k 10 200 python bench.py --steps 20 --warmup 5 --fp32-steps 0 --no-check > $OUT/rs$rs.$rep.log 2>&1 || exit $?
  done
done
