#!/bin/bash
# Static CU share for the two backward kernels (XDOT_BWD_PGRID_COLS / _ROWS: persistent grids
# walking their items) vs one workgroup per item: flash GPU tests under a persistent grid, then the
# concurrent pair (bench_flash --concurrent) and the step per setting, interleaved on one box.
set -o pipefail
T=${1:-r4pgrid}
O=gpurun_out/$T
mkdir -p $O
XDOT_BWD_PGRID_COLS=96 XDOT_BWD_PGRID_ROWS=64 timeout -k 10 300 python -u -m pytest tests/test_flash_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest_pgrid.log 2>&1 || exit $?
for rep in 1 2; do
  for cfg in "0 0" "256 256" "320 192" "384 128" "512 512"; do
    set -- $cfg
    XDOT_BWD_PGRID_COLS=$1 XDOT_BWD_PGRID_ROWS=$2 timeout -k 10 120 python benchmarks/bench_flash.py --only bwd_cols --concurrent --iters 10 > $O/pair_${1}_${2}_$rep.log 2>&1 || exit $?
    XDOT_BWD_PGRID_COLS=$1 XDOT_BWD_PGRID_ROWS=$2 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --fp32-steps 0 --no-check > $O/step_${1}_${2}_$rep.log 2>&1 || exit $?
  done
done
echo pgrid-ok
