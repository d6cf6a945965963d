#!/bin/bash
# same-box A/B of two builds on the fp32 flash kernels: fp32 tests on the new build, then
# alternating bench_flash --dtype fp32 (split family) rounds and the fp32 bench step
# usage: r3_ab32.sh TAG NEW BASE
set -o pipefail
TAG=$1; NEW=$2; BASE=$3
O=gpurun_out/$TAG
mkdir -p $O
XDOT_EXT_PATH=$NEW timeout -k 10 400 python -u -m pytest tests/test_flash_f32_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit $?
for r in 1 2; do
  for v in $BASE $NEW; do
    n=$(basename $v .so)
    XDOT_EXT_PATH=$v timeout -k 10 200 python benchmarks/bench_flash.py --dtype fp32 --iters 5 >> $O/flash_$n.log 2>&1 || exit $?
    XDOT_EXT_PATH=$v timeout -k 10 300 python bench.py --dtype fp32 --steps 5 --warmup 2 --no-check >> $O/bench_$n.log 2>&1 || exit $?
  done
done
echo ab32-ok
