#!/bin/bash
# exact-fp32 dK pass (score-buffer mode) with the forward's split model vs xdot/_C_base.so: N=1 and N=8 fp32 steps
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r6rsplit}; mkdir -p $OUT
cd $GRAFT_REPO_ROOT
for rep in 1 2 3; do
  for so in _C _C_base; do
    XDOT_EXT_PATH=$GRAFT_REPO_ROOT/xdot/$so.so timeout -k 10 300 python bench.py --dtype fp32 --steps 6 --warmup 2 --fp32-steps 0 --no-check > $OUT/n1_$so.$rep.log 2>&1 || exit $?
    echo "n1 $so $rep $(grep -o '"ms_per_step": [0-9.]*' $OUT/n1_$so.$rep.log)"
  done
done
for rep in 1 2; do
  for so in _C _C_base; do
    XDOT_EXT_PATH=$GRAFT_REPO_ROOT/xdot/$so.so timeout -k 10 300 python benchmarks/bench_rank.py --world 8 --steps 5 --warmup 2 --dtype fp32 --fp32-steps 0 --no-check > $OUT/r8_$so.$rep.log 2>&1 || exit $?
    echo "r8 $so $rep $(grep -o '"ms_per_step": [0-9.]*' $OUT/r8_$so.$rep.log)"
  done
done
