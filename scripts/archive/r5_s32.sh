#!/bin/bash
# Round 5 pass 32: closing health -- full GPU suite, smoke, default bench, masked ratio
# (interleaved), long context T = 200000 at the reference example's heads (h = 2) and h = 8
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5s32}; mkdir -p $OUT
export XDOT_EXT_PATH=$GRAFT_REPO_ROOT/xdot/_C.so
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest exit $rc" >> $OUT/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > $OUT/bench.log 2>&1 || exit $?
for rep in 1 2; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --fp32-steps 0 --no-check > $OUT/mask_zeros.$rep.log 2>&1 || exit $?
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --fp32-steps 0 --no-check --mask random > $OUT/mask_random.$rep.log 2>&1 || exit $?
done
timeout -k 10 400 python bench.py --seq-len 200000 --heads 2 --steps 3 --warmup 1 --fp32-steps 0 --no-check > $OUT/long_h2.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --seq-len 200000 --heads 8 --steps 3 --warmup 1 --fp32-steps 0 --no-check > $OUT/long_h8.log 2>&1 || exit $?
