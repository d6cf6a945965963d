#!/bin/bash
# One GPU verification pass (run via gpurun from the repo root):
#   tests marked gpu -> bench.py -> rocprofv3 kernel stats of bench.py.
# Usage: bash scripts/archive/gpu_check.sh <tag> [pytest selector] [bench args...]
# Every GPU step has its own time limit; a failing/killed step stops the chain.
set -o pipefail
TAG=${1:-run}; SEL=${2:-tests}; shift 2 2>/dev/null
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -m pytest $SEL -m gpu -q -rf > $OUT/pytest.log 2>&1
rc=$?; echo "pytest exit $rc" >> $OUT/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi   # 1 = test failures: keep going, anything else: stop
timeout -k 10 300 python bench.py "$@" > $OUT/bench.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof -o prof --output-format csv \
  -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 "$@" > $GRAFT_REPO_ROOT/$OUT/prof.log 2>&1
