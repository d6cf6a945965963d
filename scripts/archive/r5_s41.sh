#!/bin/bash
# Round 5 pass 41: wide 16-bit backward with the mask select only on partial tiles (SELB) vs the
# per-score form on every tile (XDOT_WIDE_NOSELB); unmasked and 10 % random mask
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r5s41; mkdir -p $OUT
R=$GRAFT_REPO_ROOT
XDOT_EXT_PATH=$R/xdot/_C.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_flash_wide_gpu.py > $OUT/test.log 2>&1 || exit $?
for rep in 1 2; do
  for v in _C _C_noselb; do
    for cfg in "256 3" "192 4" "160 4"; do
      set -- $cfg
      XDOT_EXT_PATH=$R/xdot/$v.so timeout -k 10 200 python benchmarks/bench_flash.py --iters 10 --D $1 --H $2 > $OUT/$v.D$1.$rep.log 2>&1 || exit $?
    done
    XDOT_EXT_PATH=$R/xdot/$v.so timeout -k 10 200 python benchmarks/bench_flash.py --iters 10 --D 256 --H 3 --mask --mask-density 0.1 > $OUT/$v.D256m.$rep.log 2>&1 || exit $?
  done
done
