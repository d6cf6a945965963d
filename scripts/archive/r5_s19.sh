#!/bin/bash
# Round 5 pass 19: how much of the bf16 flash kernels' time is exposed DMA latency?  Timing-only
# variant without the per-tile DMA waits (XDOT_AB_NOWAIT, wrong results) vs HEAD, interleaved;
# then a kernel trace of the bf16 step at HEAD
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r5s19; mkdir -p $OUT
for rep in 1 2; do
  for v in "" _nowait; do
    XDOT_EXT_PATH=$GRAFT_REPO_ROOT/xdot/_C$v.so timeout -k 10 200 python benchmarks/bench_flash.py --iters 20 > $OUT/bf16$v.$rep.log 2>&1 || exit $?
    XDOT_EXT_PATH=$GRAFT_REPO_ROOT/xdot/_C$v.so timeout -k 10 200 python benchmarks/bench_flash.py --iters 20 --R 3125 > $OUT/bf16_r3125$v.$rep.log 2>&1 || exit $?
  done
done
export XDOT_EXT_PATH=$GRAFT_REPO_ROOT/xdot/_C.so
bash $GRAFT_REPO_ROOT/scripts/gpu_prof_step.sh r5s19/step || exit $?
