#!/bin/bash
# rocprofv3 kernel trace + stats of the bf16 headline step (N=1) and of the emulated N=8 rank step,
# bf16 steps only (no fp32 companion, no numerics check).  Summaries: scripts/step_kernels.py.
set -o pipefail
TAG=${1:-profstep}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o prof \
  -- python3 $GRAFT_REPO_ROOT/bench.py --steps 4 --warmup 2 --fp32-steps 0 --no-check > $O/prof.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof8 -o prof \
  -- python3 $GRAFT_REPO_ROOT/benchmarks/bench_rank.py --world 8 --steps 6 --warmup 3 --fp32-steps 0 > $O/prof8.log 2>&1 || exit $?
echo prof-ok
