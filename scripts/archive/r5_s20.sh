#!/bin/bash
# Round 5 pass 20: column splits of the fp32 forward / row kernels from their own occupancy and
# a tile-cost model (XDOT_F32_SPLIT old = the 16-bit model, auto = model for the forward, all =
# forward + row kernel); kernels, then the fp32 steps
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r5s20; mkdir -p $OUT
export XDOT_EXT_PATH=$GRAFT_REPO_ROOT/xdot/_C.so
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread \
  tests/test_flash_f32_gpu.py tests/test_production_shape_gpu.py > $OUT/pytest.log 2>&1
rc=$?; echo "pytest exit $rc" >> $OUT/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
for sp in old auto all; do
  for m in exact split; do
    XDOT_F32_SPLIT=$sp timeout -k 10 200 python benchmarks/bench_flash.py --dtype fp32 --fp32-mode $m --iters 5 --scores > $OUT/${m}_$sp.log 2>&1 || exit $?
  done
done
for sp in old auto all; do
  XDOT_F32_SPLIT=$sp timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $OUT/bench_$sp.log 2>&1 || exit $?
done
