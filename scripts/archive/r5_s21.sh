#!/bin/bash
# Round 5 pass 21: exact-fp32 step timeline at HEAD (row-split column kernels, fp32 split model)
# and PMC passes of the exact-fp32 kernels
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r5s21; mkdir -p $OUT
export XDOT_EXT_PATH=$GRAFT_REPO_ROOT/xdot/_C.so
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --dtype fp32 --fp32-steps 0 --no-diagnostics > $OUT/prof.log 2>&1 || exit $?
FLASH_ARGS="--dtype fp32 --fp32-mode exact --scores" PMC_ARGS="--iters 2" bash $GRAFT_REPO_ROOT/scripts/pmc_head.sh r5s21/pmc || exit $?
