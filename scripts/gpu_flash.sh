#!/bin/bash
# Flash kernel numerics + timings only (fast loop while tuning a kernel).
set -e
O=gpurun_out/fl
mkdir -p $O
timeout -k 10 600 python -m pytest tests/test_flash_gpu.py -x -q -m gpu > $O/tests.log 2>&1
timeout -k 10 120 python benchmarks/bench_flash.py --mask --iters 10 > $O/flash_n1.log 2>&1
timeout -k 10 120 python benchmarks/bench_flash.py --mask --iters 20 --R 3125 > $O/flash_n8.log 2>&1
timeout -k 10 120 python benchmarks/bench_flash.py --mask --iters 10 --concurrent --only bwd_cols > $O/conc_n1.log 2>&1
echo ok
