#!/bin/bash
# gemm3 (csrc/gemm3.hip): numerics first, then timings against hipBLASLt and the v2 kernel.
set -e
O=gpurun_out/gemm3
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gemm3_gpu.py -x -v --timeout 120 --timeout-method thread -m gpu > $O/tests.log 2>&1
echo tests-ok
timeout -k 10 300 python -u benchmarks/bench_gemm.py --path v3 --cases ${CASES:-nt,nt_small,all,tn,all3,tn3} > $O/v3.log 2>&1
cat $O/v3.log
echo bench-ok
