#!/bin/bash
# Round 5 pass 13: separate dS buffer -> dV pass concurrent with the row kernel (module path)
set -o pipefail
export XDOT_EXT_PATH=$GRAFT_REPO_ROOT/xdot/_C.so
OUT=$GRAFT_REPO_ROOT/gpurun_out/r5s13; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread \
  tests/test_flash_f32_gpu.py tests/test_module_gpu.py tests/test_flash_wide_gpu.py > $OUT/pytest.log 2>&1
rc=$?; echo "pytest exit $rc" >> $OUT/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $OUT/bench.log 2>&1 || exit $?
XDOT_FP32_SCORES_DS=0 timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $OUT/bench_inplace.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --dtype fp32 --fp32-steps 0 --no-diagnostics > $OUT/prof.log 2>&1 || exit $?
exit $rc
