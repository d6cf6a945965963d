#!/bin/bash
# cols2 (software-pipelined column kernel) validation + A/B vs the plain kernel, then the headline
set -o pipefail
O=gpurun_out/${1:-r3cols}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_flash_gpu.py tests/test_module_gpu.py tests/test_graphs_gpu.py tests/test_kernels_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit $?
for r in 1 2; do
  for v in 0 1; do
    timeout -k 10 120 python benchmarks/bench_flash.py --mask --iters 10 --only bwd_cols --concurrent >> $O/cols_$v.log 2>&1 || exit $?
    timeout -k 10 120 python benchmarks/bench_flash.py --mask --iters 10 --only bwd_cols --concurrent --R 3125 >> $O/cols_$v.log 2>&1 || exit $?
  done
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --fp32-steps 0 > $O/bench_p0.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --mask random --fp32-steps 0 > $O/bench_rand.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --mask block-causal --fp32-steps 0 > $O/bench_bc.log 2>&1 || exit $?
timeout -k 10 300 python benchmarks/bench_rank.py --world 8 --steps 20 --warmup 5 > $O/rank8.log 2>&1 || exit $?
echo cols-ok
