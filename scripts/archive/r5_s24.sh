#!/bin/bash
# Round 5 pass 24: software-pipelined exact-fp32 forward (S(t+1) under the softmax of t) -- tests,
# then A/B vs the plain forward (XDOT_F32_FWD_PLAIN build), interleaved, and the step
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r5s24; mkdir -p $OUT
export XDOT_EXT_PATH=$GRAFT_REPO_ROOT/xdot/_C.so
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread \
  tests/test_flash_f32_gpu.py tests/test_production_shape_gpu.py > $OUT/pytest.log 2>&1
rc=$?; echo "pytest exit $rc" >> $OUT/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
for rep in 1 2; do
  for v in _fwdplain ""; do
    XDOT_EXT_PATH=$GRAFT_REPO_ROOT/xdot/_C$v.so timeout -k 10 200 python benchmarks/bench_flash.py --dtype fp32 --fp32-mode exact --iters 5 --scores --only fwd > $OUT/exact$v.$rep.log 2>&1 || exit $?
    XDOT_EXT_PATH=$GRAFT_REPO_ROOT/xdot/_C$v.so timeout -k 10 200 python benchmarks/bench_flash.py --dtype fp32 --fp32-mode exact --iters 5 --only fwd > $OUT/exact_nosb$v.$rep.log 2>&1 || exit $?
  done
done
for v in _fwdplain ""; do
  XDOT_EXT_PATH=$GRAFT_REPO_ROOT/xdot/_C$v.so timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $OUT/bench$v.log 2>&1 || exit $?
done
