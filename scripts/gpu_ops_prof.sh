#!/bin/bash
# rocprofv3 kernel stats + trace of one bench_ops case (emulated N=8 rank)
set -o pipefail
TAG=${1:-opsprof}; MODE=${2:-nt}; shift 2
O=gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_$MODE -o prof \
  -- python3 $GRAFT_REPO_ROOT/benchmarks/bench_ops.py --mode $MODE --iters 5 --warmup 2 "$@" > $GRAFT_REPO_ROOT/$O/$MODE.log 2>&1 || exit $?
echo prof-ok
