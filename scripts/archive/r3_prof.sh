#!/bin/bash
# tests of this round's changes + kernel traces of the N=1 step (all-False and random mask)
set -o pipefail
O=gpurun_out/${1:-r3prof}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_flash_gpu.py tests/test_module_gpu.py tests/test_ipc_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit $?
timeout -k 10 200 python benchmarks/bench_flash.py --mask --mask-density 0.1 --iters 10 > $O/flash_rand.log 2>&1 || exit $?
timeout -k 10 200 python benchmarks/bench_flash.py --mask --iters 10 > $O/flash_zero.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/p1 -o prof \
  -- python3 $GRAFT_REPO_ROOT/bench.py --steps 4 --warmup 2 --fp32-steps 0 --no-check > $GRAFT_REPO_ROOT/$O/p1.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/p1r -o prof \
  -- python3 $GRAFT_REPO_ROOT/bench.py --steps 4 --warmup 2 --fp32-steps 0 --no-check --mask random > $GRAFT_REPO_ROOT/$O/p1r.log 2>&1 || exit $?
echo prof-ok
