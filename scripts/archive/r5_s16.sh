#!/bin/bash
# Round 5 pass 16: uniform S/dS memory ops per tile (dump block for waves that own no block) so
# the compiler's vmcnt waits stay exact -- A/B vs the previous kernels (_C_prev.so); tests
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r5s16; mkdir -p $OUT
for v in "" _prev; do
  for m in exact split; do
    XDOT_EXT_PATH=$GRAFT_REPO_ROOT/xdot/_C$v.so timeout -k 10 200 python benchmarks/bench_flash.py --dtype fp32 --fp32-mode $m --iters 5 --scores > $OUT/${m}$v.log 2>&1 || exit $?
  done
done
export XDOT_EXT_PATH=$GRAFT_REPO_ROOT/xdot/_C.so
timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread \
  tests/test_flash_f32_gpu.py tests/test_production_shape_gpu.py tests/test_flash_wide_gpu.py tests/test_module_gpu.py > $OUT/pytest.log 2>&1
rc=$?; echo "pytest exit $rc" >> $OUT/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $OUT/bench.log 2>&1 || exit $?
exit $rc
