#!/bin/bash
# Round 5 pass 39: wide 16-bit forward at two workgroups per CU (D <= 256) vs one (XDOT_WIDE_OCC1)
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r5s39; mkdir -p $OUT
R=$GRAFT_REPO_ROOT
XDOT_EXT_PATH=$R/xdot/_C.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_flash_wide_gpu.py > $OUT/test.log 2>&1 || exit $?
for rep in 1 2; do
  for v in _C _C_occ1; do
    for cfg in "256 3" "192 4" "160 4" "384 2"; do
      set -- $cfg
      XDOT_EXT_PATH=$R/xdot/$v.so timeout -k 10 200 python benchmarks/bench_flash.py --iters 20 --only fwd --D $1 --H $2 > $OUT/$v.D$1.$rep.log 2>&1 || exit $?
    done
  done
done
