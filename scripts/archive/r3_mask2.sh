#!/bin/bash
# masked-path + rows-split check
set -o pipefail
O=gpurun_out/${1:-r3mask2}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_flash_gpu.py tests/test_module_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit $?
timeout -k 10 200 python benchmarks/bench_flash.py --mask --mask-density 0.1 --iters 10 > $O/flash_rand.log 2>&1 || exit $?
timeout -k 10 200 python benchmarks/bench_flash.py --mask --iters 10 > $O/flash_zero.log 2>&1 || exit $?
for m in zeros random; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --fp32-steps 0 --mask $m > $O/bench_$m.log 2>&1 || exit $?
done
timeout -k 10 300 python benchmarks/bench_rank.py --world 2 4 8 --steps 20 --warmup 5 > $O/rank.log 2>&1 || exit $?
echo mask2-ok
