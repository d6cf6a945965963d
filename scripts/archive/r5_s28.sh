#!/bin/bash
# Round 5 pass 28: split-family buffer modes after the image-layout change: S + dS buffers /
# dS only (default) / recompute; all inside bench.py's split step
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r5s28; mkdir -p $OUT
export XDOT_EXT_PATH=$GRAFT_REPO_ROOT/xdot/_C.so
for rep in 1 2; do
  XDOT_FP32_DS_ONLY=none timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $OUT/bench_sds.$rep.log 2>&1 || exit $?
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $OUT/bench_dsonly.$rep.log 2>&1 || exit $?
  XDOT_FP32_SCORES=0 timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $OUT/bench_recompute.$rep.log 2>&1 || exit $?
done
