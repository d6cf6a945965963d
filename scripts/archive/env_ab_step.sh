#!/bin/bash
# A/B of one environment switch on whole steps only: module / async-ordering / graph GPU tests
# under the B setting, then 3 alternating rounds of {bench.py N=1, bench_rank N=8}, then a
# kernel trace of the emulated N=8 rank step under B.
# usage: env_ab_step.sh TAG VAR valA valB
set -o pipefail
TAG=$1; VAR=$2; A=$3; B=$4
O=gpurun_out/$TAG
mkdir -p $O
env $VAR=$B timeout -k 10 500 python -u -m pytest tests/test_module_gpu.py tests/test_async_comm_gpu.py tests/test_graphs_gpu.py \
  tests/test_layouts.py tests/test_ipc_gpu.py -q -m gpu --timeout 200 --timeout-method thread -rf > $O/tests_B.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/tests_B.log
if [ $rc -ne 0 ]; then exit $rc; fi
for r in 1 2 3; do
  for v in $A $B; do
    tag=$([ $v == $A ] && echo A || echo B)
    env $VAR=$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 >> $O/step_$tag.log 2>&1 || exit $?
    env $VAR=$v timeout -k 10 200 python benchmarks/bench_rank.py --world 8 --steps 20 --warmup 5 >> $O/step_$tag.log 2>&1 || exit $?
  done
done
cd /tmp && export TMPDIR=/tmp
export $VAR=$B
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/prof8 -o prof \
  -- python3 $GRAFT_REPO_ROOT/benchmarks/bench_rank.py --world 8 --steps 6 --warmup 3 > $GRAFT_REPO_ROOT/$O/prof8.log 2>&1 || exit $?
echo ab-ok
