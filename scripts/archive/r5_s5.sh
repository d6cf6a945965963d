#!/bin/bash
# Round 5 pass 5: AGPR-pinned accumulators (fp32 exact + split cols/rows kernels), grouped fp32 GEMM
set -o pipefail
OUT=gpurun_out/r5s5; mkdir -p $OUT
timeout -k 10 200 python benchmarks/bench_flash.py --dtype fp32 --fp32-mode exact --iters 5 --scores > $OUT/scores.log 2>&1 || exit $?
timeout -k 10 200 python benchmarks/bench_flash.py --dtype fp32 --fp32-mode exact --iters 5 > $OUT/exact.log 2>&1 || exit $?
timeout -k 10 200 python benchmarks/bench_flash.py --dtype fp32 --fp32-mode split --iters 5 > $OUT/split.log 2>&1 || exit $?
timeout -k 10 300 python benchmarks/bench_gemm.py --dtype fp32 --cases proj,proj_dx,wgrad,nt_wide,all3,tn3 --iters 5 > $OUT/gemm.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread \
  tests/test_flash_f32_gpu.py tests/test_production_shape_gpu.py tests/test_gemm_f32_gpu.py tests/test_flash_gpu.py tests/test_flash_wide_gpu.py > $OUT/pytest.log 2>&1
rc=$?; echo "pytest exit $rc" >> $OUT/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
FLASH_ARGS="--dtype fp32 --fp32-mode exact --scores" bash scripts/pmc_head.sh r5s5/pmc_f32sb || exit $?
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $OUT/bench.log 2>&1 || exit $?
exit $rc
