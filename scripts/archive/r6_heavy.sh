#!/bin/bash
# exact-fp32 forward on the head-heavy grid: fp32 GPU tests, then the exact-fp32 step A/B
# (XDOT_F32_HEAVY=1 vs 0, 3 interleaved reps) and a kernel trace of the new step
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r6heavy}; mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_flash_f32_gpu.py tests/test_module_gpu.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
bash scripts/ab_step.sh ${1:-r6heavy}/ab 3 "--dtype fp32 --steps 10 --warmup 3" xdot/_C.so:XDOT_F32_HEAVY=1 xdot/_C.so:XDOT_F32_HEAVY=0 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/fp32 -o prof \
  -- python3 $GRAFT_REPO_ROOT/bench.py --dtype fp32 --steps 3 --warmup 2 --fp32-steps 0 --no-check > $OUT/fp32.log 2>&1 || exit $?
echo heavy-ok
