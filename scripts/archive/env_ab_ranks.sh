#!/bin/bash
# A/B of one environment switch over the whole rank-shape range: module GPU tests under B, then
# 3 alternating rounds of {bench.py N=1, bench_rank N=2/4/8 (emulated per-rank steps)}.
# usage: env_ab_ranks.sh TAG VAR valA valB
set -o pipefail
TAG=$1; VAR=$2; A=$3; B=$4
O=gpurun_out/$TAG
mkdir -p $O
env $VAR=$B timeout -k 10 400 python -u -m pytest tests/test_module_gpu.py tests/test_async_comm_gpu.py -q -m gpu \
  --timeout 200 --timeout-method thread -rf > $O/tests_B.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/tests_B.log
if [ $rc -ne 0 ]; then exit $rc; fi
for r in 1 2 3; do
  for v in $A $B; do
    tag=$([ $v == $A ] && echo A || echo B)
    env $VAR=$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 >> $O/step_$tag.log 2>&1 || exit $?
    env $VAR=$v timeout -k 10 300 python benchmarks/bench_rank.py --world 2 4 8 --steps 20 --warmup 5 >> $O/step_$tag.log 2>&1 || exit $?
  done
done
echo ab-ok
