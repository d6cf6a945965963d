#!/bin/bash
# Round 5 pass 11: select-free softmax loops in the fp32 / split column kernels (mask fix-up only
# on partially masked tiles), S prefetch depth 1
set -o pipefail
export XDOT_EXT_PATH=$GRAFT_REPO_ROOT/xdot/_C.so
OUT=$GRAFT_REPO_ROOT/gpurun_out/r5s11; mkdir -p $OUT
for m in exact split; do
  timeout -k 10 200 python benchmarks/bench_flash.py --dtype fp32 --fp32-mode $m --iters 5 --scores > $OUT/$m.log 2>&1 || exit $?
  timeout -k 10 200 python benchmarks/bench_flash.py --dtype fp32 --fp32-mode $m --iters 5 --scores --mask --mask-density 0.1 > $OUT/${m}_mask.log 2>&1 || exit $?
done
timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread \
  tests/test_flash_f32_gpu.py tests/test_production_shape_gpu.py tests/test_gemm_f32_gpu.py > $OUT/pytest.log 2>&1
rc=$?; echo "pytest exit $rc" >> $OUT/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $OUT/bench.log 2>&1 || exit $?
exit $rc
