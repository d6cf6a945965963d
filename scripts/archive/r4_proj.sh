#!/bin/bash
# Projection GEMM (csrc/gemm_proj.hip): GPU tests, hipBLASLt vs xdot per shape, then a step A/B on
# one box over the fused node / side-stream weight gradients / projection kernel at the three
# step shapes (N=1 T=25000, N=1 T=5000, emulated N=8 rank), then the module GPU tests.
set -o pipefail
T=${1:-r4proj}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_proj_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest_proj.log 2>&1 || exit $?
timeout -k 10 300 python benchmarks/micro/linear_host.py --quick > $O/linear_host.log 2>&1 || exit $?
for cfg in "XDOT_FUSED_MODULE=1" "XDOT_FUSED_MODULE=0" "XDOT_WGRAD_SIDE=0" "XDOT_PROJ=0"; do
  tag=$(echo $cfg | tr '=' '_')
  env $cfg timeout -k 10 200 python bench.py --steps 20 --warmup 5 --fp32-steps 0 --no-check >> $O/n1_$tag.log 2>&1 || exit $?
  env $cfg timeout -k 10 200 python bench.py --seq-len 5000 --steps 50 --warmup 10 --fp32-steps 0 --no-check >> $O/t5k_$tag.log 2>&1 || exit $?
  env $cfg timeout -k 10 200 python benchmarks/bench_rank.py --world 8 --steps 30 --warmup 5 --fp32-steps 0 >> $O/r8_$tag.log 2>&1 || exit $?
done
timeout -k 10 300 python benchmarks/host_step_profile.py --world 8 --steps 40 > $O/host8.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_module_gpu.py tests/test_graphs_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest_module.log 2>&1 || exit $?
echo proj-ok
