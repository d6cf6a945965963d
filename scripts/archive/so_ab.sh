#!/bin/bash
# A/B of compile-time variants built by scripts/build_variant.sh: flash GPU tests under each
# variant, then 3 alternating rounds of bench_flash (one kernel, N=1 and the N=8 rank shape).
# usage: so_ab.sh TAG KERNEL VARIANT... (VARIANT "base" = xdot/_C.so)
set -o pipefail
TAG=$1; KER=$2; shift 2
O=gpurun_out/$TAG
mkdir -p $O
so() { if [ "$1" == "base" ]; then echo xdot/_C.so; else echo xdot/_C_$1.so; fi; }
for v in "$@"; do
  XDOT_EXT_PATH=$(so $v) timeout -k 10 300 python -u -m pytest tests/test_flash_gpu.py -q -m gpu --timeout 120 --timeout-method thread -x > $O/tests_$v.log 2>&1 || exit $?
done
echo tests-ok
for r in 1 2 3; do
  for v in "$@"; do
    XDOT_EXT_PATH=$(so $v) timeout -k 10 120 python benchmarks/bench_flash.py --mask --iters 10 --only $KER >> $O/$v.log 2>&1 || exit $?
    XDOT_EXT_PATH=$(so $v) timeout -k 10 120 python benchmarks/bench_flash.py --mask --iters 10 --only $KER --R 3125 >> $O/$v.log 2>&1 || exit $?
  done
done
echo ab-ok
