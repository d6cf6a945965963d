#!/bin/bash
# Round 5 pass 9: persistent 256x256 LDS-DMA fp32 GEMM (csrc/gemm2_f32.hip) tests + A/B vs the
# 128x128 kernel (path 1) and hipBLASLt; PMC of the fp32 score-buffer kernels
set -o pipefail
export XDOT_EXT_PATH=$GRAFT_REPO_ROOT/xdot/_C.so
OUT=$GRAFT_REPO_ROOT/gpurun_out/r5s9; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gemm_f32_gpu.py > $OUT/pytest_gemm.log 2>&1 || exit $?
for path in auto v1 v2; do
  timeout -k 10 300 python benchmarks/bench_gemm.py --dtype fp32 --path $path --cases proj,proj_dx,wgrad,nt_wide,all3,tn3 --iters 5 > $OUT/gemm_$path.log 2>&1 || exit $?
done
FLASH_ARGS="--dtype fp32 --fp32-mode exact --scores" bash scripts/pmc_head.sh r5s9/pmc_f32sb || exit $?
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $OUT/bench.log 2>&1 || exit $?
