#!/bin/bash
# masked-path check: flash/module GPU tests, kernel times with a 10 % random mask, headline step
# with all-False / random / block-causal masks
set -o pipefail
O=gpurun_out/${1:-r3mask}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_flash_gpu.py tests/test_module_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit $?
timeout -k 10 200 python benchmarks/bench_flash.py --mask --mask-density 0.1 --iters 10 > $O/flash_rand.log 2>&1 || exit $?
timeout -k 10 200 python benchmarks/bench_flash.py --mask --iters 10 > $O/flash_zero.log 2>&1 || exit $?
for m in zeros random block-causal; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --fp32-steps 0 --mask $m > $O/bench_$m.log 2>&1 || exit $?
done
timeout -k 10 200 python benchmarks/bench_flash.py --mask --mask-density 0.1 --iters 10 --R 3125 > $O/flash_rand8.log 2>&1 || exit $?
for ns in 2 3 4 6; do
  timeout -k 10 200 python benchmarks/bench_flash.py --mask --iters 10 --R 3125 --only bwd_rows --concurrent --nsplit $ns > $O/rows8_ns$ns.log 2>&1 || exit $?
done
echo mask-ok
