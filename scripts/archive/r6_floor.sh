#!/bin/bash
# Exact-fp32 step next to the bare fp32 MFMA rate ON THE SAME BOX (the clock-limited floor of
# the six-product step: profiles/r6_fp32.md §2): microbench, step, microbench, step
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r6floor}; mkdir -p $O
cd $GRAFT_REPO_ROOT
for i in 1 2; do
  timeout -k 10 120 ./benchmarks/micro/mfma_shape f32 > $O/mfma_$i.log 2>&1 || exit $?
  timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --fp32-steps 10 --fp32-warmup 3 > $O/bench_$i.log 2>&1 || exit $?
  tail -1 $O/bench_$i.log
done
echo floor-ok
