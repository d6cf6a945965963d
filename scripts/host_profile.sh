#!/bin/bash
# Host-side (Python) profile of the headline step: cProfile over 30 steps at N=1 and at the
# emulated N=8 rank; top functions by own and cumulative time.
set -o pipefail
O=gpurun_out/${1:-hostprof}
mkdir -p $O
timeout -k 10 300 python -m cProfile -o $O/n1.prof bench.py --steps 30 --warmup 5 > $O/n1.log 2>&1 || exit $?
timeout -k 10 300 python -m cProfile -o $O/n8.prof benchmarks/bench_rank.py --world 8 --steps 30 --warmup 5 > $O/n8.log 2>&1 || exit $?
echo host-ok
