#!/bin/bash
# Round 5 pass 25: wide-head kernels with split counts from their own occupancy (row splits of
# both column passes, column splits of forward / row side) -- tests, then A/B (XDOT_WIDE_SPLIT=0
# = previous behaviour vs auto) at the reference example's heads (D = 384, h = 2) and D = 256 h = 3
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r5s25; mkdir -p $OUT
export XDOT_EXT_PATH=$GRAFT_REPO_ROOT/xdot/_C.so
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_flash_wide_gpu.py > $OUT/pytest.log 2>&1
rc=$?; echo "pytest exit $rc" >> $OUT/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
for sp in 0 auto; do
  XDOT_WIDE_SPLIT=$sp timeout -k 10 200 python benchmarks/bench_flash.py --D 384 --H 2 --iters 10 > $OUT/d384_$sp.log 2>&1 || exit $?
  XDOT_WIDE_SPLIT=$sp timeout -k 10 200 python benchmarks/bench_flash.py --D 256 --H 3 --iters 10 > $OUT/d256_$sp.log 2>&1 || exit $?
  XDOT_WIDE_SPLIT=$sp timeout -k 10 300 python benchmarks/bench_flash.py --D 384 --H 2 --iters 3 --dtype fp32 --fp32-mode exact --scores > $OUT/d384_f32_$sp.log 2>&1 || exit $?
done
