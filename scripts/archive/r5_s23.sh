#!/bin/bash
# Round 5 pass 23: S / dS stores split around the MFMA block (LDS writes before it, transposed
# global stores after) -- A/B vs the previous build, interleaved; tests
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r5s23; mkdir -p $OUT
for rep in 1 2; do
  for v in _prev ""; do
    for m in exact split; do
      XDOT_EXT_PATH=$GRAFT_REPO_ROOT/xdot/_C$v.so timeout -k 10 200 python benchmarks/bench_flash.py --dtype fp32 --fp32-mode $m --iters 5 --scores > $OUT/${m}$v.$rep.log 2>&1 || exit $?
    done
  done
done
export XDOT_EXT_PATH=$GRAFT_REPO_ROOT/xdot/_C.so
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_flash_f32_gpu.py > $OUT/pytest.log 2>&1
rc=$?; echo "pytest exit $rc" >> $OUT/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
for v in _prev ""; do
  XDOT_EXT_PATH=$GRAFT_REPO_ROOT/xdot/_C$v.so timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $OUT/bench$v.log 2>&1 || exit $?
done
