#!/bin/bash
# Round 5 pass 22: dS-only buffer mode (XDOT_FP32_DS_ONLY) -- tests, kernels with / without the
# score buffer, then the fp32 steps with the mode off / split family / both families
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r5s22; mkdir -p $OUT
export XDOT_EXT_PATH=$GRAFT_REPO_ROOT/xdot/_C.so
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread \
  tests/test_flash_f32_gpu.py > $OUT/pytest.log 2>&1
rc=$?; echo "pytest exit $rc" >> $OUT/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
for m in split exact; do
  timeout -k 10 200 python benchmarks/bench_flash.py --dtype fp32 --fp32-mode $m --iters 5 > $OUT/${m}_recompute.log 2>&1 || exit $?
done
for ds in none split all; do
  XDOT_FP32_DS_ONLY=$ds timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $OUT/bench_$ds.log 2>&1 || exit $?
done
