#!/bin/bash
# Round 5 pass 1: exact-fp32 score-buffer mode (tests, kernel timings, bench).
set -o pipefail
OUT=gpurun_out/r5s1; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_flash_f32_gpu.py tests/test_production_shape_gpu.py > $OUT/pytest.log 2>&1
rc=$?; echo "pytest exit $rc" >> $OUT/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python benchmarks/bench_flash.py --dtype fp32 --fp32-mode exact --iters 5 > $OUT/flash_f32.log 2>&1 || exit $?
timeout -k 10 200 python benchmarks/bench_flash.py --dtype fp32 --fp32-mode exact --iters 5 --scores > $OUT/flash_f32_scores.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $OUT/bench.log 2>&1 || exit $?
# 2 gloo ranks sharing the one GPU: the N>1 diagnostics fields
timeout -k 10 300 python bench.py --gpus 2 --backend gloo --seq-len 5000 --steps 5 --warmup 2 --fp32-steps 0 > $OUT/gloo2.log 2>&1 || exit $?
exit $rc
