#!/bin/bash
# Projection kernel A/B round 2: fragment prefetch (GP_PRE), priority off, 256x128 8-wave tiles at
# large M (GP_HUGE); correctness of the new configurations first.
set -o pipefail
T=${1:-r4projab2}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_proj_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest_base.log 2>&1 || exit $?
for v in huge hugepre pre; do
  XDOT_EXT_PATH=xdot/_C_$v.so timeout -k 10 300 python -u -m pytest tests/test_proj_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest_$v.log 2>&1 || exit $?
done
for v in base pre noprio huge hugepre; do
  if [ $v == base ]; then P=""; else P="xdot/_C_$v.so"; fi
  XDOT_EXT_PATH=$P timeout -k 10 300 python benchmarks/micro/linear_host.py --quick > $O/lh_$v.log 2>&1 || exit $?
done
echo projab2-ok
