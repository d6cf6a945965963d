#!/bin/bash
# Paired weight-gradient launch: tests, then steps (interleaved with XDOT_WGRAD=0 for reference).
set -o pipefail
T=${1:-r4pair}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_proj_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
for rep in 1 2; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --fp32-steps 0 --no-check > $O/n1_$rep.log 2>&1 || exit $?
  timeout -k 10 200 python benchmarks/bench_rank.py --world 8 --steps 30 --warmup 5 --fp32-steps 0 > $O/r8_$rep.log 2>&1 || exit $?
done
timeout -k 10 600 python -u -m pytest tests/test_module_gpu.py tests/test_graphs_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest_module.log 2>&1 || exit $?
echo pair-ok
