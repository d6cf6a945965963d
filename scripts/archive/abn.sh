#!/bin/bash
# Time several extension builds (abtest/<V>.so for V in $VARIANTS) in one GPU session,
# alternating, 2 rounds; args go to benchmarks/bench_flash.py.
O=gpurun_out/abn
mkdir -p $O
rm -f $O/*.log
for r in 1 2; do
  for v in ${VARIANTS:-A B}; do
    XDOT_EXT_PATH=abtest/$v.so timeout -k 10 120 python benchmarks/bench_flash.py "$@" >> $O/$v.log 2>&1 || exit 1
  done
done
echo ok
