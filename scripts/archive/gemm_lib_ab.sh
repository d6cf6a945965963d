#!/bin/bash
# Library route of xdot.gemm (XDOT_GEMM_LIB=1, default) vs xdot kernels only (0): GEMM + ops
# numerics, bench_gemm through the op dispatcher, and the distributed-op configs 3/4.
set -o pipefail
O=gpurun_out/${1:-gemm_lib}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gemm2_gpu.py tests/test_kernels_gpu.py tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu > $O/tests.log 2>&1 || exit $?
echo tests-ok
for v in 1 0; do
  XDOT_GEMM_LIB=$v timeout -k 10 300 python benchmarks/bench_gemm.py --cases nt,nt_small,all,tn,all3,tn3 > $O/gemm_lib$v.log 2>&1 || exit $?
  XDOT_GEMM_LIB=$v timeout -k 10 300 python benchmarks/bench_gemm.py --dtype fp32 --cases nt_small,all3,tn3 > $O/gemm_f32_lib$v.log 2>&1 || exit $?
  for m in nt all; do
    for dt in bf16 fp32; do
      XDOT_GEMM_LIB=$v timeout -k 10 200 python benchmarks/bench_ops.py --mode $m --T 25000 --offset 32 --emulate 8 --dtype $dt --iters 5 > $O/c3_${m}_${dt}_lib$v.log 2>&1 || exit $?
      XDOT_GEMM_LIB=$v timeout -k 10 200 python benchmarks/bench_ops.py --mode $m --T 75000 --dtype $dt --iters 3 > $O/n1_${m}_${dt}_lib$v.log 2>&1 || exit $?
    done
  done
  XDOT_GEMM_LIB=$v timeout -k 10 200 python benchmarks/bench_ops.py --mode leftT_fb --T 12500 --emulate 8 --dtype bf16 --iters 5 > $O/c4_lib$v.log 2>&1 || exit $?
done
echo bench-ok
