#!/bin/bash
# Round 5 pass 51: closing rocprofv3 kernel traces of the three N=1 steps at HEAD (bf16, exact
# fp32, split fp32) and of the reference example's heads (D = 384, h = 2, bf16)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r5s51; mkdir -p $O
export XDOT_EXT_PATH=$GRAFT_REPO_ROOT/xdot/_C.so
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/bf16 -o prof \
  -- python3 $GRAFT_REPO_ROOT/bench.py --steps 4 --warmup 2 --fp32-steps 0 --no-check > $O/bf16.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/exact -o prof \
  -- python3 $GRAFT_REPO_ROOT/bench.py --dtype fp32 --steps 3 --warmup 1 --fp32-steps 0 --no-check > $O/exact.log 2>&1 || exit $?
XDOT_FP32_MODE=split timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/split -o prof \
  -- python3 $GRAFT_REPO_ROOT/bench.py --dtype fp32 --steps 3 --warmup 1 --fp32-steps 0 --no-check > $O/split.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/h2 -o prof \
  -- python3 $GRAFT_REPO_ROOT/bench.py --heads 2 --steps 4 --warmup 2 --fp32-steps 0 --no-check > $O/h2.log 2>&1 || exit $?
echo prof-ok
