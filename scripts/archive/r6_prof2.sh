#!/bin/bash
# fp32 step kernel trace, fp32 kernel PMC (score-buffer mode), emulated N=8 rank kernel trace + table
set -o pipefail
TAG=${1:-r6prof2}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/fp32 -o prof \
  -- python3 $GRAFT_REPO_ROOT/bench.py --dtype fp32 --steps 3 --warmup 2 --fp32-steps 0 --no-check > $O/fp32.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rank8 -o prof \
  -- python3 $GRAFT_REPO_ROOT/benchmarks/bench_rank.py --world 8 --steps 6 --warmup 3 --fp32-steps 0 > $O/rank8.log 2>&1 || exit $?
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python benchmarks/bench_rank.py --world 2 4 8 --steps 20 --warmup 5 --fp32-steps 0 --no-check > $O/ranks.log 2>&1 || exit $?
FLASH_ARGS="--dtype fp32 --scores" bash scripts/pmc_head.sh $TAG/pmc || exit $?
echo prof2-ok
