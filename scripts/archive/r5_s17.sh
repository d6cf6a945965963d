#!/bin/bash
# Round 5 pass 17: row splits of the fp32 column kernels (XDOT_CSPLIT) against the last-round
# tail -- tests, then kernel A/B (1 = unsplit vs auto), then the step
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r5s17; mkdir -p $OUT
export XDOT_EXT_PATH=$GRAFT_REPO_ROOT/xdot/_C.so
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread \
  tests/test_flash_f32_gpu.py > $OUT/pytest.log 2>&1
rc=$?; echo "pytest exit $rc" >> $OUT/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
for cs in 1 auto; do
  for m in exact split; do
    XDOT_CSPLIT=$cs timeout -k 10 200 python benchmarks/bench_flash.py --dtype fp32 --fp32-mode $m --iters 5 --scores > $OUT/${m}_cs$cs.log 2>&1 || exit $?
  done
done
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $OUT/bench.log 2>&1 || exit $?
XDOT_CSPLIT=1 timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $OUT/bench_cs1.log 2>&1 || exit $?
