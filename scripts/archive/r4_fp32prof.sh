#!/bin/bash
# Kernel trace of the exact-fp32 N=1 step (the reference's precision) and of the split-bf16 one.
set -o pipefail
T=${1:-r4fp32prof}
O=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/exact -o prof \
  -- python3 $GRAFT_REPO_ROOT/bench.py --dtype fp32 --steps 3 --warmup 1 --no-check > $O/exact.log 2>&1 || exit $?
echo fp32prof-ok
