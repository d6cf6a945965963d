#!/bin/bash
# Quick check of a step-level change: given GPU tests, N=1 bench, emulated N=8 rank (3 runs) and a
# kernel trace of the emulated N=8 step.  usage: gpu_quick8.sh TAG [pytest files...]
set -o pipefail
TAG=$1; shift
O=gpurun_out/$TAG
mkdir -p $O
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -u -m pytest "$@" -m gpu -q --timeout 120 --timeout-method thread -rf > $O/pytest.log 2>&1 || exit $?
fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || exit $?
for r in 1 2 3; do
  timeout -k 10 300 python benchmarks/bench_rank.py --world 8 --steps 20 --warmup 5 >> $O/rank.log 2>&1 || exit $?
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof8 -o prof \
  -- python3 $GRAFT_REPO_ROOT/benchmarks/bench_rank.py --world 8 --steps 6 --warmup 3 > $GRAFT_REPO_ROOT/$O/prof8.log 2>&1 || exit $?
echo quick-ok
