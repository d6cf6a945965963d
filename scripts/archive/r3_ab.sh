#!/bin/bash
# same-box A/B of two builds (XDOT_EXT_PATH): flash tests on the new build, then alternating
# rounds of kernel timings (N=1 and the N=8 rank shape) and the headline step.
# usage: r3_ab.sh TAG NEW BASE   (NEW/BASE: .so paths)
set -o pipefail
TAG=$1; NEW=$2; BASE=$3
O=gpurun_out/$TAG
mkdir -p $O
XDOT_EXT_PATH=$NEW timeout -k 10 400 python -u -m pytest tests/test_flash_gpu.py tests/test_module_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit $?
for r in 1 2; do
  for v in $BASE $NEW; do
    n=$(basename $v .so)
    XDOT_EXT_PATH=$v timeout -k 10 200 python benchmarks/bench_flash.py --mask --iters 10 >> $O/flash_$n.log 2>&1 || exit $?
    XDOT_EXT_PATH=$v timeout -k 10 200 python benchmarks/bench_flash.py --mask --iters 10 --R 3125 >> $O/flash8_$n.log 2>&1 || exit $?
    XDOT_EXT_PATH=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --fp32-steps 0 --no-check >> $O/bench_$n.log 2>&1 || exit $?
  done
done
echo ab-ok
