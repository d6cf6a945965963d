#!/bin/bash
# Round 5 pass 42: (a) partial-tile mask select extended to the D = 384 dV pass and the fp32 wide
# kernels that keep their registers, A/B against XDOT_WIDE_NOSELB; (b) the 16-bit D = 256 dV pass
# at two workgroups per CU, A/B against XDOT_WIDE_COLS_OCC1
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r5s42; mkdir -p $OUT
R=$GRAFT_REPO_ROOT
XDOT_EXT_PATH=$R/xdot/_C.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_flash_wide_gpu.py > $OUT/test.log 2>&1 || exit $?
for rep in 1 2; do
  for v in _C _C_cocc1; do
    XDOT_EXT_PATH=$R/xdot/$v.so timeout -k 10 200 python benchmarks/bench_flash.py --iters 10 --D 256 --H 3 --only bwd_cols > $OUT/$v.D256.$rep.log 2>&1 || exit $?
    XDOT_EXT_PATH=$R/xdot/$v.so timeout -k 10 200 python benchmarks/bench_flash.py --iters 10 --D 256 --H 3 --only bwd_cols --mask --mask-density 0.1 > $OUT/$v.D256m.$rep.log 2>&1 || exit $?
  done
  for v in _C _C_noselb; do
    XDOT_EXT_PATH=$R/xdot/$v.so timeout -k 10 200 python benchmarks/bench_flash.py --iters 10 --D 384 --H 2 > $OUT/$v.D384.$rep.log 2>&1 || exit $?
    XDOT_EXT_PATH=$R/xdot/$v.so timeout -k 10 300 python benchmarks/bench_flash.py --iters 5 --D 256 --H 3 --dtype fp32 --fp32-mode exact > $OUT/$v.f32D256.$rep.log 2>&1 || exit $?
    XDOT_EXT_PATH=$R/xdot/$v.so timeout -k 10 300 python benchmarks/bench_flash.py --iters 5 --D 384 --H 2 --dtype fp32 --fp32-mode exact > $OUT/$v.f32D384.$rep.log 2>&1 || exit $?
  done
done
