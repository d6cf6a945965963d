#!/bin/bash
# Default bench (numerics check, bf16, both fp32 modes) after keeping library weight gradients
# off the side stream; then the fused-node GPU tests.
set -o pipefail
T=${1:-r4fix}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 300 python bench.py --trace > $O/bench.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_module_gpu.py tests/test_gemm3_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
echo fix-ok
