#!/bin/bash
# Row-side backward column splits at N=1 (the occupancy model picks 3 -> fp32 partials + a sum
# pass) and at the N=8 rank, interleaved on one box; plus the host numbers after the GradSync /
# fused-backward trims.
set -o pipefail
T=${1:-r4split}
O=gpurun_out/$T
mkdir -p $O
for rep in 1 2; do
  for s in 0 1 2 4; do
    XDOT_ROWS_SPLIT=$s timeout -k 10 200 python bench.py --steps 20 --warmup 5 --fp32-steps 0 --no-check > $O/n1_s${s}_$rep.log 2>&1 || exit $?
  done
done
for s in 0 4 8; do
  XDOT_ROWS_SPLIT=$s timeout -k 10 200 python benchmarks/bench_rank.py --world 8 --steps 30 --warmup 5 --fp32-steps 0 > $O/r8_s${s}.log 2>&1 || exit $?
done
timeout -k 10 200 python bench.py --seq-len 5000 --steps 50 --warmup 10 --fp32-steps 0 --no-check > $O/t5k.log 2>&1 || exit $?
timeout -k 10 300 python benchmarks/host_step_profile.py --world 8 --steps 40 > $O/host8.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_module_gpu.py tests/test_async_comm_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
echo split-ok
