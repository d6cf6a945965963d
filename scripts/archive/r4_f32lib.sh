#!/bin/bash
# Exact-fp32 products: library fp32 GEMM (default XDOT_GEMM_LIB) vs the hand-written exact kernel
# with K slabs (XDOT_GEMM_LIB=0), BASELINE configs 3-4 as one rank of 8, interleaved twice.
set -o pipefail
T=${1:-r4f32lib}
O=gpurun_out/$T; mkdir -p $O
for rep in 1 2; do
  for lib in d 0; do
    for m in leftT_fb rightT_fb full_fb; do
      if [ $lib = d ]; then E=""; else E="XDOT_GEMM_LIB=0"; fi
      env $E timeout -k 10 200 python benchmarks/bench_ops.py --mode $m --T 12500 --emulate 8 --dtype fp32 --iters 10 --no-local 2>&1 | grep '"mode"' | sed "s/^/lib=$lib /" >> $O/ab.log || exit $?
    done
    for m in nt all; do
      if [ $lib = d ]; then E=""; else E="XDOT_GEMM_LIB=0"; fi
      env $E timeout -k 10 200 python benchmarks/bench_ops.py --mode $m --T 25000 --offset 32 --emulate 8 --dtype fp32 --iters 10 --no-local 2>&1 | grep '"mode"' | sed "s/^/lib=$lib /" >> $O/ab.log || exit $?
    done
  done
done
echo f32lib-ok
