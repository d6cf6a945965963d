#!/bin/bash
# Round 5 pass 4: score-buffer store variants (A/B via XDOT_EXT_PATH), fp32 GEMM PMC, remaining tests.
set -o pipefail
OUT=gpurun_out/r5s4; mkdir -p $OUT
for v in "" _nopipe _sbdirect _nods _nosload; do
  XDOT_EXT_PATH=xdot/_C$v.so timeout -k 10 200 python benchmarks/bench_flash.py --dtype fp32 --fp32-mode exact --iters 5 --scores > $OUT/scores$v.log 2>&1 || exit $?
done
timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread \
  tests/test_flash_wide_gpu.py tests/test_production_shape_gpu.py tests/test_flash_f32_gpu.py > $OUT/pytest.log 2>&1
rc=$?; echo "pytest exit $rc" >> $OUT/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
PMC_SCRIPT=benchmarks/bench_gemm.py PMC_ARGS="--dtype fp32 --cases nt_wide,proj --iters 3 --warmup 1" bash scripts/pmc_head.sh r5s4/pmc_gemm || exit $?
FLASH_ARGS="--dtype fp32 --fp32-mode exact --scores" bash scripts/pmc_head.sh r5s4/pmc_f32sb || exit $?
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $OUT/bench.log 2>&1 || exit $?
exit $rc
