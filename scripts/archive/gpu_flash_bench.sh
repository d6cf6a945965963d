#!/bin/bash
# flash kernel timings (N=1 and N=8 per-rank shapes) + the headline bench at N=1
set -e
O=gpurun_out/${1:-fb}
mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_flash_gpu.py tests/test_module_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu > $O/tests.log 2>&1
timeout -k 10 200 python benchmarks/bench_flash.py --mask --iters 10 --concurrent > $O/n1.log 2>&1
timeout -k 10 200 python benchmarks/bench_flash.py --mask --iters 10 --R 3125 --concurrent > $O/n8.log 2>&1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1
timeout -k 10 300 python benchmarks/bench_rank.py --world 8 --steps 20 --warmup 5 > $O/rank8.log 2>&1
echo fb-ok
