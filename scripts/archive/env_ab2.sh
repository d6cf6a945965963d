#!/bin/bash
# A/B of one environment switch: flash/module GPU tests under the B setting, then 3 alternating
# rounds of {bench_flash at N=1 and the N=8 rank shape, bench.py N=1, bench_rank N=8}.
# usage: env_ab2.sh TAG VAR valA valB [bench_flash kernel: fwd|bwd_cols|bwd_rows]
set -o pipefail
TAG=$1; VAR=$2; A=$3; B=$4; KER=${5:-bwd_cols}
O=gpurun_out/$TAG
mkdir -p $O
env $VAR=$B timeout -k 10 400 python -u -m pytest tests/test_flash_gpu.py tests/test_module_gpu.py tests/test_long_context_gpu.py \
  -q -m gpu --timeout 120 --timeout-method thread -rf > $O/tests_B.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/tests_B.log
if [ $rc -ne 0 ]; then exit $rc; fi
for r in 1 2 3; do
  for v in $A $B; do
    tag=$([ $v == $A ] && echo A || echo B)
    env $VAR=$v timeout -k 10 120 python benchmarks/bench_flash.py --mask --iters 10 --only $KER >> $O/$tag.log 2>&1 || exit $?
    env $VAR=$v timeout -k 10 120 python benchmarks/bench_flash.py --mask --iters 10 --only $KER --R 3125 >> $O/$tag.log 2>&1 || exit $?
    env $VAR=$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 >> $O/step_$tag.log 2>&1 || exit $?
    env $VAR=$v timeout -k 10 200 python benchmarks/bench_rank.py --world 8 --steps 20 --warmup 5 >> $O/step_$tag.log 2>&1 || exit $?
  done
done
echo ab-ok
