#!/bin/bash
# Weight-gradient slab cost model: tests, sweep (auto vs fixed S), steps.
set -o pipefail
T=${1:-r4ws2}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_proj_gpu.py -x -q --timeout 120 --timeout-method thread -k wgrad > $O/pytest.log 2>&1 || exit $?
timeout -k 10 300 python benchmarks/micro/wgrad_splits.py > $O/ws.log 2>&1 || exit $?
for rep in 1 2; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --fp32-steps 0 --no-check > $O/n1_$rep.log 2>&1 || exit $?
  timeout -k 10 200 python benchmarks/bench_rank.py --world 8 --steps 30 --warmup 5 --fp32-steps 0 > $O/r8_$rep.log 2>&1 || exit $?
done
echo ws2-ok
