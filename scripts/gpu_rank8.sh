#!/bin/bash
# Emulated per-rank steps (N = 2, 4, 8 on one GPU) + kernel timeline of the N=8 rank step.
set -e
O=gpurun_out/rank8
mkdir -p $O
timeout -k 10 300 python benchmarks/bench_rank.py --world 2 4 8 --steps 20 --warmup 5 > $O/rank.log 2>&1
echo rank-ok
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o prof \
  -- python3 $GRAFT_REPO_ROOT/benchmarks/bench_rank.py --world 8 --steps 10 --warmup 3 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1
echo prof-ok
