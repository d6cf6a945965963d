#!/bin/bash
# Round 5 pass 27: split-bf16 (x3) images in the bf16 kernels' swizzled row-major layout, the
# transposed operands through ds_read_b64_tr_b16 (no 2-byte transposed LDS writes) -- tests, then
# A/B vs the previous build (interleaved) and the step
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r5s27; mkdir -p $OUT
export XDOT_EXT_PATH=$GRAFT_REPO_ROOT/xdot/_C.so
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_flash_f32_gpu.py > $OUT/pytest.log 2>&1
rc=$?; echo "pytest exit $rc" >> $OUT/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
for rep in 1 2; do
  for v in _prev ""; do
    XDOT_EXT_PATH=$GRAFT_REPO_ROOT/xdot/_C$v.so timeout -k 10 200 python benchmarks/bench_flash.py --dtype fp32 --fp32-mode split --iters 5 --scores > $OUT/scores$v.$rep.log 2>&1 || exit $?
    XDOT_EXT_PATH=$GRAFT_REPO_ROOT/xdot/_C$v.so timeout -k 10 200 python benchmarks/bench_flash.py --dtype fp32 --fp32-mode split --iters 5 > $OUT/recompute$v.$rep.log 2>&1 || exit $?
  done
done
for v in _prev ""; do
  XDOT_EXT_PATH=$GRAFT_REPO_ROOT/xdot/_C$v.so timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $OUT/bench$v.log 2>&1 || exit $?
done
