#!/bin/bash
# round-3 baseline at HEAD: flash kernel timings, headline bench (zeros / random mask), fp32 step
set -e
O=gpurun_out/${1:-r3base}
mkdir -p $O
timeout -k 10 200 python benchmarks/bench_flash.py --mask --iters 10 --concurrent > $O/n1.log 2>&1
timeout -k 10 200 python benchmarks/bench_flash.py --mask --iters 10 --R 3125 --concurrent > $O/n8.log 2>&1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --mask random > $O/bench_rand.log 2>&1
timeout -k 10 300 python benchmarks/bench_rank.py --world 8 --steps 20 --warmup 5 > $O/rank8.log 2>&1
echo base-ok
