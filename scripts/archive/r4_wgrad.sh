#!/bin/bash
# Weight-gradient kernel (csrc/gemm_wgrad.hip): GPU tests, micro-benchmark against hipBLASLt and
# the gemm3 split-K route, then the steps with it on / off (XDOT_WGRAD), interleaved.
set -o pipefail
T=${1:-r4wgrad}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_proj_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
timeout -k 10 300 python benchmarks/micro/linear_host.py --quick > $O/lh.log 2>&1 || exit $?
for rep in 1 2; do
  for w in 1 0; do
    XDOT_WGRAD=$w timeout -k 10 200 python bench.py --steps 20 --warmup 5 --fp32-steps 0 --no-check > $O/n1_w${w}_$rep.log 2>&1 || exit $?
    XDOT_WGRAD=$w timeout -k 10 200 python benchmarks/bench_rank.py --world 8 --steps 30 --warmup 5 --fp32-steps 0 > $O/r8_w${w}_$rep.log 2>&1 || exit $?
  done
done
timeout -k 10 600 python -u -m pytest tests/test_module_gpu.py tests/test_gemm3_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest_module.log 2>&1 || exit $?
echo wgrad-ok
