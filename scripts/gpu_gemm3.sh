#!/bin/bash
# gemm3 (csrc/gemm3.hip): numerics first, then timings against hipBLASLt (and rotation off).
set -e
O=gpurun_out/gemm3
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gemm3_gpu.py -x -v --timeout 120 --timeout-method thread -m gpu > $O/tests.log 2>&1
echo tests-ok
tail -1 $O/tests.log
C=${CASES:-nt,nt_small,all,tn,all3,tn3}
timeout -k 10 300 python -u benchmarks/bench_gemm.py --path v3 --cases $C > $O/v3.log 2>&1
XDOT_GEMM3_ROTATE=0 timeout -k 10 300 python -u benchmarks/bench_gemm.py --path v3 --cases $C > $O/v3_norot.log 2>&1
grep case $O/v3.log; echo "-- rotation off"; grep case $O/v3_norot.log
echo bench-ok
