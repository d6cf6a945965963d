#!/bin/bash
# Quick GPU iteration loop: flash/module GPU tests, kernel timings (N=1 and N=8 per-rank shapes),
# the headline bench at N=1 and the emulated N=8 per-rank step.  Stops at the first failure.
set -e
O=gpurun_out/quick
mkdir -p $O
timeout -k 10 600 python -m pytest tests/test_flash_gpu.py tests/test_module_gpu.py -x -q -m gpu > $O/tests.log 2>&1
timeout -k 10 120 python benchmarks/bench_flash.py --mask --iters 10 > $O/flash_n1.log 2>&1
timeout -k 10 120 python benchmarks/bench_flash.py --mask --iters 20 --R 3125 > $O/flash_n8.log 2>&1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench1.log 2>&1
timeout -k 10 300 python benchmarks/bench_rank.py --world 8 --steps 20 --warmup 5 > $O/rank8.log 2>&1
echo ok
