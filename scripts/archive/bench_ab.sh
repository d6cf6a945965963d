#!/bin/bash
# A/B of one environment switch on the headline bench in one GPU session (alternating runs).
# usage: bench_ab.sh VAR valA valB [rounds] -- extra bench.py args
VAR=$1; A=$2; B=$3; N=${4:-3}; shift 4; [ "$1" = "--" ] && shift
O=gpurun_out/benchab
mkdir -p $O
rm -f $O/*.log
for r in $(seq $N); do
  for v in $A $B; do
    env $VAR=$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 "$@" >> $O/$v.log 2>&1 || exit 1
  done
done
for v in $A $B; do echo "$VAR=$v: $(grep -o '"value": [0-9.]*' $O/$v.log | awk '{print $2}' | tr '\n' ' ')"; done
