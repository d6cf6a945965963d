#!/bin/bash
# 8-lane bf16 δ prep: flash GPU tests, then a bf16 N=1 step trace and an emulated N=8 one
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r6prep}; mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_flash_gpu.py tests/test_production_shape_gpu.py tests/test_flash_wide_gpu.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/n1 -o prof \
  -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --fp32-steps 0 > $OUT/n1.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/rank8 -o prof \
  -- python3 $GRAFT_REPO_ROOT/benchmarks/bench_rank.py --world 8 --steps 10 --warmup 3 --fp32-steps 0 --no-check > $OUT/rank8.log 2>&1 || exit $?
echo prep-ok
