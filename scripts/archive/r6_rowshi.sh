#!/bin/bash
# (A/B) N=1 bf16 step with the row kernel on the high-priority stream (XDOT_AB_ROWS_HI=1) vs HEAD
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r6rowshi}; mkdir -p $OUT
cd $GRAFT_REPO_ROOT
for rep in 1 2 3; do
  for v in 0 1; do
    XDOT_AB_ROWS_HI=$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 --fp32-steps 0 > $OUT/n1_v$v.$rep.log 2>&1 || exit $?
  done
done
echo rowshi-ok
