#!/bin/bash
# Step-level A/B of a compile-time variant (scripts/build_variant.sh) against xdot/_C.so: GPU
# flash/module tests on the default build, then 3 alternating rounds of bench.py N=1 and the
# emulated N=8 rank.  usage: so_step_ab.sh TAG VARIANT
set -o pipefail
TAG=$1; V=$2
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_flash_gpu.py tests/test_module_gpu.py -q -m gpu --timeout 120 --timeout-method thread -x > $O/tests.log 2>&1 || exit $?
echo tests-ok
for r in 1 2 3; do
  for so in xdot/_C.so xdot/_C_$V.so; do
    tag=$([ $so == xdot/_C.so ] && echo base || echo $V)
    XDOT_EXT_PATH=$so timeout -k 10 200 python bench.py --steps 20 --warmup 5 >> $O/step_$tag.log 2>&1 || exit $?
    XDOT_EXT_PATH=$so timeout -k 10 200 python benchmarks/bench_rank.py --world 8 --steps 20 --warmup 5 >> $O/step_$tag.log 2>&1 || exit $?
  done
done
echo ab-ok
