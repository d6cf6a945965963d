#!/bin/bash
# Round 5 pass 36: bf16 forward with its row sums on the matrix pipe (ones block in the PV
# product, XDOT_FWD_MFMA_SUM build) -- flash tests on the variant, then A/B vs HEAD (interleaved)
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r5s36; mkdir -p $OUT
XDOT_EXT_PATH=$GRAFT_REPO_ROOT/xdot/_C_msum.so timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread \
  tests/test_flash_gpu.py tests/test_production_shape_gpu.py > $OUT/pytest.log 2>&1
rc=$?; echo "pytest exit $rc" >> $OUT/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
for rep in 1 2 3; do
  for v in "" _msum; do
    XDOT_EXT_PATH=$GRAFT_REPO_ROOT/xdot/_C$v.so timeout -k 10 200 python benchmarks/bench_flash.py --iters 20 --only fwd > $OUT/fwd$v.$rep.log 2>&1 || exit $?
    XDOT_EXT_PATH=$GRAFT_REPO_ROOT/xdot/_C$v.so timeout -k 10 200 python benchmarks/bench_flash.py --iters 20 --only fwd --R 3125 > $OUT/fwd8$v.$rep.log 2>&1 || exit $?
  done
done
for v in "" _msum; do
  XDOT_EXT_PATH=$GRAFT_REPO_ROOT/xdot/_C$v.so timeout -k 10 200 python bench.py --steps 20 --warmup 5 --fp32-steps 0 --no-check > $OUT/bench$v.log 2>&1 || exit $?
done
