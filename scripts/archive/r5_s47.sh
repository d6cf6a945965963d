#!/bin/bash
# Round 5 pass 47: LDS operand reads 2 (HEAD) / 3 / 4 MFMAs ahead in the one-workgroup-per-CU
# wide kernels (XDOT_WIDE_LA)
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r5s47; mkdir -p $OUT
R=$GRAFT_REPO_ROOT
for rep in 1 2; do
  for v in _C _C_la3 _C_la4; do
    for cfg in "256 3" "384 2"; do
      set -- $cfg
      XDOT_EXT_PATH=$R/xdot/$v.so timeout -k 10 200 python benchmarks/bench_flash.py --iters 10 --D $1 --H $2 > $OUT/$v.D$1.$rep.log 2>&1 || exit $?
    done
  done
done
