#!/bin/bash
# Round 5 pass 50: pipelined wide dQ pass, each score chain spread over three MFMA gaps, vs the
# plain pass (XDOT_WIDE_NODQPIPE)
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r5s50; mkdir -p $OUT
R=$GRAFT_REPO_ROOT
XDOT_EXT_PATH=$R/xdot/_C.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_flash_wide_gpu.py > $OUT/test.log 2>&1 || exit $?
for rep in 1 2; do
  for v in _C _C_nodqpipe; do
    for cfg in "256 3" "192 4" "160 4"; do
      set -- $cfg
      XDOT_EXT_PATH=$R/xdot/$v.so timeout -k 10 200 python benchmarks/bench_flash.py --iters 10 --D $1 --H $2 --only bwd_cols > $OUT/$v.D$1.$rep.log 2>&1 || exit $?
    done
  done
done
