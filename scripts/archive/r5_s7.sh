#!/bin/bash
# Round 5 pass 7: split-bf16 score-buffer mode (fwd+S, dV pass, dQ pass, rows from dS); per-kernel
# rocprof stats of both fp32 families with the score buffer
set -o pipefail
export XDOT_EXT_PATH=$GRAFT_REPO_ROOT/xdot/_C.so
OUT=$GRAFT_REPO_ROOT/gpurun_out/r5s7; mkdir -p $OUT
timeout -k 10 200 python benchmarks/bench_flash.py --dtype fp32 --fp32-mode split --iters 5 --scores > $OUT/split_scores.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread \
  tests/test_flash_f32_gpu.py tests/test_production_shape_gpu.py tests/test_module_gpu.py > $OUT/pytest.log 2>&1
rc=$?; echo "pytest exit $rc" >> $OUT/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp
for m in exact split; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$m -o run -- python3 $GRAFT_REPO_ROOT/benchmarks/bench_flash.py --dtype fp32 --fp32-mode $m --iters 3 --scores > $OUT/prof_$m.log 2>&1 || exit $?
done
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $OUT/bench.log 2>&1 || exit $?
exit $rc
