#!/bin/bash
# Round 5 pass 38: where the random-mask cost goes -- bf16 kernels with no mask vs a 10 % random
# mask (T = R = 25000 and the N=8 rank shape)
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r5s38; mkdir -p $OUT
export XDOT_EXT_PATH=$GRAFT_REPO_ROOT/xdot/_C.so
for rep in 1 2; do
  timeout -k 10 200 python benchmarks/bench_flash.py --iters 20 > $OUT/nomask.$rep.log 2>&1 || exit $?
  timeout -k 10 200 python benchmarks/bench_flash.py --iters 20 --mask --mask-density 0.1 > $OUT/mask10.$rep.log 2>&1 || exit $?
  timeout -k 10 200 python benchmarks/bench_flash.py --iters 20 --R 3125 > $OUT/nomask8.$rep.log 2>&1 || exit $?
  timeout -k 10 200 python benchmarks/bench_flash.py --iters 20 --R 3125 --mask --mask-density 0.1 > $OUT/mask10_8.$rep.log 2>&1 || exit $?
done
