#!/bin/bash
# Round 5 pass 14: swizzled S/dS transpose tile (A/B vs _noswz), fp32 GEMM DMA issue placement
# (A/B _iss1 staggered by wave half, _iss2 spread), tests
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r5s14; mkdir -p $OUT
for v in "" _noswz; do
  for m in exact split; do
    XDOT_EXT_PATH=$GRAFT_REPO_ROOT/xdot/_C$v.so timeout -k 10 200 python benchmarks/bench_flash.py --dtype fp32 --fp32-mode $m --iters 5 --scores > $OUT/${m}$v.log 2>&1 || exit $?
  done
done
for v in "" _iss1 _iss2; do
  XDOT_EXT_PATH=$GRAFT_REPO_ROOT/xdot/_C$v.so timeout -k 10 300 python benchmarks/bench_gemm.py --dtype fp32 --path v2 --cases nt_wide,all3,tn3,wgrad --iters 5 > $OUT/gemm$v.log 2>&1 || exit $?
done
export XDOT_EXT_PATH=$GRAFT_REPO_ROOT/xdot/_C.so
timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread \
  tests/test_flash_f32_gpu.py tests/test_gemm_f32_gpu.py tests/test_production_shape_gpu.py > $OUT/pytest.log 2>&1
rc=$?; echo "pytest exit $rc" >> $OUT/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $OUT/bench.log 2>&1 || exit $?
exit $rc
