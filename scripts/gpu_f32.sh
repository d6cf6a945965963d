#!/bin/bash
# fp32 headline numbers: fused fp32 path (N=1, emulated N=8), the materialised fp32 path for
# comparison, and a rocprofv3 kernel-stats pass of the fused fp32 step.
set -o pipefail
TAG=${1:-f32}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python bench.py --dtype fp32 --steps 5 --warmup 2 > $O/bench_f32.log 2>&1 || exit $?
timeout -k 10 300 python benchmarks/bench_rank.py --world 8 --dtype fp32 --steps 5 --warmup 2 > $O/rank_f32.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --dtype fp32 --impl materialized --steps 3 --warmup 1 > $O/bench_f32_mat.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o prof \
  -- python3 $GRAFT_REPO_ROOT/bench.py --dtype fp32 --steps 2 --warmup 1 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || exit $?
echo f32-ok
