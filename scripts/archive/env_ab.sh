#!/bin/bash
# A/B of one environment switch in one GPU session: flash GPU tests under both settings, then
# alternating bench_flash timings.  usage: env_ab.sh VAR valA valB -- <bench_flash args>
VAR=$1; A=$2; B=$3; shift 4
O=gpurun_out/envab
mkdir -p $O
rm -f $O/*.log
for v in $A $B; do
  env $VAR=$v timeout -k 10 300 python -m pytest tests/test_flash_gpu.py tests/test_long_context_gpu.py -x -q -m gpu > $O/tests_$v.log 2>&1 || { echo "tests failed under $VAR=$v"; exit 1; }
done
for r in 1 2; do
  for v in $A $B; do
    env $VAR=$v timeout -k 10 120 python benchmarks/bench_flash.py "$@" >> $O/$v.log 2>&1 || exit 1
  done
done
echo ok
