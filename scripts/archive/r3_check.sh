#!/bin/bash
# quick GPU check: optimizer/graph tests + headline bench (zeros / random / block-causal mask)
set -e
O=gpurun_out/${1:-r3check}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_graphs_gpu.py tests/test_kernels_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --mask random --fp32-steps 0 > $O/bench_rand.log 2>&1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --mask block-causal --fp32-steps 0 > $O/bench_bc.log 2>&1
timeout -k 10 300 python benchmarks/bench_rank.py --world 8 --steps 20 --warmup 5 > $O/rank8.log 2>&1
echo check-ok
