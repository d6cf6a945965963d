#!/bin/bash
# rocprofv3 kernel traces (+ stats) of the N=1 bf16 step, the N=1 exact-fp32 step and the emulated
# N=8 rank step (bf16).  Summaries: scripts/step_kernels.py <dir>/prof*/prof_kernel_trace.csv
set -o pipefail
TAG=${1:-r6prof}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/bf16 -o prof \
  -- python3 $GRAFT_REPO_ROOT/bench.py --steps 4 --warmup 2 --fp32-steps 0 --no-check > $O/bf16.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/fp32 -o prof \
  -- python3 $GRAFT_REPO_ROOT/bench.py --dtype fp32 --steps 3 --warmup 2 --fp32-steps 0 --no-check > $O/fp32.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rank8 -o prof \
  -- python3 $GRAFT_REPO_ROOT/benchmarks/bench_rank.py --world 8 --steps 6 --warmup 3 --fp32-steps 0 > $O/rank8.log 2>&1 || exit $?
echo prof-ok
