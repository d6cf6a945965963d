#!/bin/bash
# Round 5 pass 6: score-buffer column side as two passes (dV from S, then dQ at 2 waves / SIMD);
# fp32 GEMM predicate-free interior loads + 2-tile-ahead prefetch (A/B vs 1-ahead: _C_pf1.so)
set -o pipefail
export XDOT_EXT_PATH=xdot/_C.so
OUT=gpurun_out/r5s6; mkdir -p $OUT
timeout -k 10 200 python benchmarks/bench_flash.py --dtype fp32 --fp32-mode exact --iters 5 --scores > $OUT/scores.log 2>&1 || exit $?
for v in "" _pf1; do
  XDOT_EXT_PATH=xdot/_C$v.so timeout -k 10 300 python benchmarks/bench_gemm.py --dtype fp32 --cases proj,proj_dx,nt_wide,all3,tn3 --iters 5 > $OUT/gemm$v.log 2>&1 || exit $?
done
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread \
  tests/test_flash_f32_gpu.py tests/test_production_shape_gpu.py tests/test_gemm_f32_gpu.py > $OUT/pytest.log 2>&1
rc=$?; echo "pytest exit $rc" >> $OUT/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/benchmarks/bench_flash.py --dtype fp32 --fp32-mode exact --iters 3 --scores > $GRAFT_REPO_ROOT/$OUT/prof.log 2>&1 || exit $?
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $OUT/bench.log 2>&1 || exit $?
exit $rc
