#!/bin/bash
# Round 5 pass 44: wide LDS-DMA piece offsets precomputed once per lane (packed, 2 per register)
# vs recomputed at every issue (XDOT_WIDE_NOPK); the D = 256 dV pass at one workgroup per CU
# (XDOT_WIDE_COLS_OCC1) on the same build for reference
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r5s44; mkdir -p $OUT
R=$GRAFT_REPO_ROOT
XDOT_EXT_PATH=$R/xdot/_C.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_flash_wide_gpu.py > $OUT/test.log 2>&1 || exit $?
for rep in 1 2; do
  for v in _C _C_nopk _C_cocc1; do
    XDOT_EXT_PATH=$R/xdot/$v.so timeout -k 10 200 python benchmarks/bench_flash.py --iters 10 --D 256 --H 3 > $OUT/$v.D256.$rep.log 2>&1 || exit $?
    XDOT_EXT_PATH=$R/xdot/$v.so timeout -k 10 200 python benchmarks/bench_flash.py --iters 10 --D 384 --H 2 > $OUT/$v.D384.$rep.log 2>&1 || exit $?
    XDOT_EXT_PATH=$R/xdot/$v.so timeout -k 10 200 python benchmarks/bench_flash.py --iters 10 --D 192 --H 4 > $OUT/$v.D192.$rep.log 2>&1 || exit $?
  done
done
