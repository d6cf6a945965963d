#!/bin/bash
# HIP-graph captured step: GPU test, then eager vs graph (2 alternating rounds) at N=1 T=25000,
# T=5000 (BASELINE config 2) and the emulated N=8 rank.
set -o pipefail
O=gpurun_out/${1:-graph}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_graphs_gpu.py tests/test_optim.py -q -m gpu --timeout 200 --timeout-method thread -x > $O/tests.log 2>&1 || exit $?
echo tests-ok
for r in 1 2; do
  for g in "" "--graph"; do
    t=$([ -z "$g" ] && echo eager || echo graph)
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 $g >> $O/n1_$t.log 2>&1 || exit $?
    timeout -k 10 200 python bench.py --seq-len 5000 --steps 50 --warmup 10 $g >> $O/t5k_$t.log 2>&1 || exit $?
    timeout -k 10 200 python benchmarks/bench_rank.py --world 8 --steps 20 --warmup 5 $g >> $O/n8_$t.log 2>&1 || exit $?
  done
done
echo bench-ok
