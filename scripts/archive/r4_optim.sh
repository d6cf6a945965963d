#!/bin/bash
# Lean FusedAdamW.step (no profiler wrapper unless observed): optimizer / graph GPU tests, then
# the host-bound shapes (T=5000 N=1, emulated N=8 rank host profile).
set -o pipefail
T=${1:-r4optim}
O=gpurun_out/$T; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_graphs_gpu.py tests/test_kernels_gpu.py tests/test_optim.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
for r in 1 2 3; do
  timeout -k 10 200 python bench.py --seq-len 5000 --steps 50 --warmup 10 --fp32-steps 0 --no-check 2>&1 | grep '"metric"' | sed 's/^/lean /' >> $O/t5k.log || exit $?
  timeout -k 10 200 python benchmarks/micro/optim_hooked.py --seq-len 5000 --steps 50 --warmup 10 --fp32-steps 0 --no-check 2>&1 | grep '"metric"' | sed 's/^/hooked /' >> $O/t5k.log || exit $?
done
timeout -k 10 300 python benchmarks/host_step_profile.py --world 8 --steps 40 > $O/host8.log 2>&1 || exit $?
timeout -k 10 300 python benchmarks/host_step_profile.py --seq-len 5000 --steps 40 > $O/host1_5k.log 2>&1 || exit $?
echo optim-ok
