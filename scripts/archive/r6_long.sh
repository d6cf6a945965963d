#!/bin/bash
# T = 200000 (BASELINE config 5): bf16 steps at h = 2 (the reference example's D = 384) and h = 8,
# the exact-fp32 step at h = 8 (recompute path: the score buffer would be 1.28 TB)
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r6long}; mkdir -p $OUT
timeout -k 10 400 python bench.py --seq-len 200000 --heads 2 --steps 3 --warmup 1 --fp32-steps 0 --no-check > $OUT/long_h2.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --seq-len 200000 --heads 8 --steps 3 --warmup 1 --fp32-steps 0 --no-check > $OUT/long_h8.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --dtype fp32 --seq-len 200000 --heads 8 --steps 2 --warmup 1 --fp32-steps 0 --no-check > $OUT/long_f32_h8.log 2>&1 || exit $?
echo long-ok
