#!/bin/bash
# Forward row sums on packed P (v_dot2c) vs HEAD's scalar adds: flash GPU tests, standalone fwd
# A/B interleaved (xdot/_C_rowsum.so = HEAD flash_fwd.hip), then the fp32-step bisect.
set -o pipefail
T=${1:-r4dot2}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_flash_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest_flash.log 2>&1 || exit $?
for i in 1 2 3; do
  timeout -k 10 120 python benchmarks/bench_flash.py --only fwd --iters 50 > $O/fwd_new_$i.log 2>&1 || exit $?
  XDOT_EXT_PATH=xdot/_C_rowsum.so timeout -k 10 120 python benchmarks/bench_flash.py --only fwd --iters 50 > $O/fwd_old_$i.log 2>&1 || exit $?
done
timeout -k 10 120 python benchmarks/bench_flash.py --only fwd --R 3125 --iters 50 > $O/fwd8_new.log 2>&1 || exit $?
XDOT_EXT_PATH=xdot/_C_rowsum.so timeout -k 10 120 python benchmarks/bench_flash.py --only fwd --R 3125 --iters 50 > $O/fwd8_old.log 2>&1 || exit $?
echo dot2-ok
bash scripts/r4_fp32dbg.sh $T/dbg
