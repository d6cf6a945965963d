#!/bin/bash
# One GPU pass: gpu tests -> bench N=1 -> emulated per-rank N=2/4/8 -> rocprofv3 kernel stats
# of bench.py (N=1) and a kernel trace of the emulated N=8 rank step.  Each GPU step has its
# own time limit; anything but "tests failed" (pytest exit 1) stops the chain.
set -o pipefail
TAG=${1:-s4}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -rf > $O/pytest.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || exit $?
timeout -k 10 300 python benchmarks/bench_rank.py --world 2 4 8 --steps 20 --warmup 5 > $O/rank.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o prof \
  -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof8 -o prof \
  -- python3 $GRAFT_REPO_ROOT/benchmarks/bench_rank.py --world 8 --steps 10 --warmup 3 > $GRAFT_REPO_ROOT/$O/prof8.log 2>&1 || exit $?
echo session-ok
