#!/bin/bash
# XDOT_WGRAD_SIDE A/B at HEAD: N=1 bf16 step (3 reps) and the emulated N=8 rank (2 reps), interleaved
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r6wside}; mkdir -p $OUT
cd $GRAFT_REPO_ROOT
for rep in 1 2 3; do
  for w in 0 1; do
    XDOT_WGRAD_SIDE=$w timeout -k 10 200 python bench.py --steps 20 --warmup 5 --fp32-steps 0 --no-check > $OUT/n1_w$w.$rep.log 2>&1 || exit $?
  done
done
for rep in 1 2; do
  for w in 0 1; do
    XDOT_WGRAD_SIDE=$w timeout -k 10 300 python benchmarks/bench_rank.py --world 8 --steps 20 --warmup 5 --fp32-steps 0 --no-check > $OUT/r8_w$w.$rep.log 2>&1 || exit $?
  done
done
echo wside-ok
