#!/bin/bash
# Round 5 pass 46: is LDS-DMA latency exposed in the wide kernels?  Timing-only build without
# the per-tile vmcnt(0) waits (XDOT_AB_NOWAIT: results wrong, timing valid) vs HEAD
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r5s46; mkdir -p $OUT
R=$GRAFT_REPO_ROOT
for rep in 1 2; do
  for v in _C _C_nowait; do
    for cfg in "256 3" "384 2"; do
      set -- $cfg
      XDOT_EXT_PATH=$R/xdot/$v.so timeout -k 10 200 python benchmarks/bench_flash.py --iters 10 --D $1 --H $2 > $OUT/$v.D$1.$rep.log 2>&1 || exit $?
    done
  done
done
