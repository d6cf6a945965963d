#!/bin/bash
# Side-stream weight gradients revisited after the host trims (inline backward, one
# linear_backward per layer, grouped bucket all-reduce): N=1 and the emulated N=8 rank, interleaved;
# then the RCCL API test.
set -o pipefail
T=${1:-r4side2}
O=gpurun_out/$T
mkdir -p $O
for rep in 1 2; do
  for s in 0 1; do
    XDOT_WGRAD_SIDE=$s timeout -k 10 200 python bench.py --steps 20 --warmup 5 --fp32-steps 0 --no-check > $O/n1_side${s}_$rep.log 2>&1 || exit $?
    XDOT_WGRAD_SIDE=$s timeout -k 10 200 python benchmarks/bench_rank.py --world 8 --steps 30 --warmup 5 --fp32-steps 0 > $O/r8_side${s}_$rep.log 2>&1 || exit $?
  done
done
timeout -k 10 200 python -u -m pytest tests/test_rccl_gpu.py -x -q --timeout 150 --timeout-method thread > $O/pytest_rccl.log 2>&1 || exit $?
echo side2-ok
