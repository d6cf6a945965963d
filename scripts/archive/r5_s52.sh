#!/bin/bash
# Round 5 pass 52: split-fp32 mode keeps its projections on the exact-fp32 GEMM kernels (was: the
# library's fp32 GEMM); tests + split / exact steps
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r5s52; mkdir -p $OUT
export XDOT_EXT_PATH=$GRAFT_REPO_ROOT/xdot/_C.so
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_flash_f32_gpu.py tests/test_proj_gpu.py tests/test_gemm3_gpu.py tests/test_production_shape_gpu.py > $OUT/test.log 2>&1 || exit $?
for rep in 1 2; do
  XDOT_FP32_MODE=split timeout -k 10 300 python bench.py --dtype fp32 --steps 5 --warmup 2 --fp32-steps 0 --no-check > $OUT/split.$rep.log 2>&1 || exit $?
  XDOT_F32_PROJ=0 XDOT_FP32_MODE=split timeout -k 10 300 python bench.py --dtype fp32 --steps 5 --warmup 2 --fp32-steps 0 --no-check > $OUT/split_lib.$rep.log 2>&1 || exit $?
done
timeout -k 10 300 python bench.py > $OUT/bench.log 2>&1 || exit $?
