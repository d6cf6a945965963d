#!/bin/bash
# round 3 GEMM pass: full GPU suite, GEMM benchmarks on the default (auto) path in bf16 and fp32
# against torch.matmul, then the headline bench.
set -o pipefail
O=gpurun_out/r3g
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -u benchmarks/bench_gemm.py --cases nt,nt_small,nt_rank8,all,tn,all3,tn3 > $O/bf16.log 2>&1 || exit 1
timeout -k 10 300 python -u benchmarks/bench_gemm.py --dtype fp32 --iters 5 --cases nt_small,nt_wide,all3,tn3 > $O/fp32.log 2>&1 || exit 1
XDOT_FP32_MODE=exact timeout -k 10 300 python -u benchmarks/bench_gemm.py --dtype fp32 --iters 5 --cases nt_small,all3 > $O/fp32_exact.log 2>&1 || exit 1
grep case $O/bf16.log $O/fp32.log $O/fp32_exact.log
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1 || exit 1
tail -1 $O/bench.log
