#!/bin/bash
# FusedAdamW: kernel GPU tests, then the optimizer step time, vector vs scalar kernel (3 rounds).
set -o pipefail
O=gpurun_out/${1:-adam}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_graphs_gpu.py -q -m gpu -k "adamw or graph" \
  --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
for r in 1 2 3; do
  timeout -k 10 120 python benchmarks/bench_optim.py >> $O/optim.log 2>&1 || exit $?
  XDOT_EXT_PATH=xdot/_C_adamscalar.so timeout -k 10 120 python benchmarks/bench_optim.py >> $O/optim.log 2>&1 || exit $?
done
echo adam-ok
