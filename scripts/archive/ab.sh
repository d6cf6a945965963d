#!/bin/bash
# A/B timing of two extension builds in one GPU session: abtest/A.so vs abtest/B.so,
# alternating runs of benchmarks/bench_flash.py (args passed through).
O=gpurun_out/ab
mkdir -p $O
rm -f $O/*.log
for r in 1 2 3; do
  for v in A B; do
    XDOT_EXT_PATH=abtest/$v.so timeout -k 10 120 python benchmarks/bench_flash.py "$@" >> $O/$v.log 2>&1 || exit 1
  done
done
echo ok
