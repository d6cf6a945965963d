#!/bin/bash
# GEMM v2 check: numerics (v2 + v1 regression), then timings vs torch.matmul.
set -e
O=gpurun_out/gemm
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gemm2_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu > $O/tests.log 2>&1
XDOT_GEMM2_PERSIST_KT=0 timeout -k 10 300 python -u -m pytest tests/test_gemm2_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu > $O/tests_np.log 2>&1
echo tests-ok
XDOT_GEMM2_PERSIST_KT=0 timeout -k 10 300 python benchmarks/bench_gemm.py > $O/v2_np.log 2>&1
XDOT_GEMM2_PERSIST_KT=0 XDOT_GEMM2_ISS=0 timeout -k 10 300 python benchmarks/bench_gemm.py > $O/v2_np0.log 2>&1
echo bench-ok
