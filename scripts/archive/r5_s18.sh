#!/bin/bash
# Round 5 pass 18: row splits of the pipelined 16-bit column kernel -- tests, kernel A/B
# (XDOT_CSPLIT=1 vs auto) at T = R = 25000 and at the N=8 rank shape, then the step
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r5s18; mkdir -p $OUT
export XDOT_EXT_PATH=$GRAFT_REPO_ROOT/xdot/_C.so
timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread \
  tests/test_flash_gpu.py tests/test_flash_f32_gpu.py tests/test_module_gpu.py tests/test_production_shape_gpu.py > $OUT/pytest.log 2>&1
rc=$?; echo "pytest exit $rc" >> $OUT/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
for cs in 1 auto; do
  XDOT_CSPLIT=$cs timeout -k 10 200 python benchmarks/bench_flash.py --iters 10 > $OUT/bf16_cs$cs.log 2>&1 || exit $?
  XDOT_CSPLIT=$cs timeout -k 10 200 python benchmarks/bench_flash.py --iters 10 --R 3125 > $OUT/bf16_r3125_cs$cs.log 2>&1 || exit $?
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench.log 2>&1 || exit $?
XDOT_CSPLIT=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench_cs1.log 2>&1 || exit $?
