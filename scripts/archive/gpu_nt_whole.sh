#!/bin/bash
# Whole-shard nt as one GEMM over all T columns: GEMM + ops GPU tests, then emulated N=8 nt
# (whole shard, offset 32) and N=1, bf16 and fp32.
set -o pipefail
O=gpurun_out/${1:-nt_whole}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gemm2_gpu.py tests/test_ops_gpu.py tests/test_module_gpu.py -q -m gpu --timeout 300 --timeout-method thread -x > $O/tests.log 2>&1 || exit $?
echo tests-ok
for dt in bf16 fp32; do
  timeout -k 10 200 python benchmarks/bench_ops.py --mode nt --T 25000 --emulate 8 --dtype $dt --iters 5 > $O/nt8_$dt.log 2>&1 || exit $?
  timeout -k 10 200 python benchmarks/bench_ops.py --mode nt --T 25000 --emulate 8 --dtype $dt --iters 5 --offset 32 > $O/nt8_o32_$dt.log 2>&1 || exit $?
  timeout -k 10 200 python benchmarks/bench_ops.py --mode nt --T 25000 --emulate 8 --dtype $dt --iters 5 --schedule ring --no-local > $O/nt8_ring_$dt.log 2>&1 || exit $?
done
echo bench-ok
