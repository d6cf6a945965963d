#!/bin/bash
# Round 5 pass 56: the 16-bit D = 160 wide row side at two workgroups per CU (XDOT_WIDE_ROWS_OCC2)
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r5s56; mkdir -p $OUT
R=$GRAFT_REPO_ROOT
XDOT_EXT_PATH=$R/xdot/_C_rocc2.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_flash_wide_gpu.py > $OUT/test.log 2>&1 || exit $?
for rep in 1 2; do
  for v in _C _C_rocc2; do
    XDOT_EXT_PATH=$R/xdot/$v.so timeout -k 10 200 python benchmarks/bench_flash.py --iters 10 --D 160 --H 4 --only bwd_rows > $OUT/$v.D160.$rep.log 2>&1 || exit $?
  done
done
