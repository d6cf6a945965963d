#!/bin/bash
# Round 5 pass 55: wide LDS-DMA pieces issued as runs (one M0 setup per <= 5 pieces, as the narrow
# kernels) vs one asm block per piece (XDOT_WIDE_NORUN); wide tests on the new build
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r5s55; mkdir -p $OUT
R=$GRAFT_REPO_ROOT
XDOT_EXT_PATH=$R/xdot/_C.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_flash_wide_gpu.py > $OUT/test.log 2>&1 || exit $?
for rep in 1 2; do
  for v in _C _C_norun; do
    for cfg in "256 3" "384 2"; do
      set -- $cfg
      XDOT_EXT_PATH=$R/xdot/$v.so timeout -k 10 200 python benchmarks/bench_flash.py --iters 10 --D $1 --H $2 > $OUT/$v.D$1.$rep.log 2>&1 || exit $?
    done
  done
done
