#!/bin/bash
# Session 2c: the session-2b pass (default bench with stage tracing, then the host / rank / ring /
# fp32-config measurements) after the stream fix, then the module and gemm3 GPU tests.
set -o pipefail
T=${1:-r4s2c}
bash scripts/r4_s2b.sh $T || exit $?
timeout -k 10 600 python -u -m pytest tests/test_module_gpu.py tests/test_gemm3_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1 || exit $?
echo s2c-ok
