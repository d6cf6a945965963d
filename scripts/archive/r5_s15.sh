#!/bin/bash
# Round 5 pass 15: fp32 trprod read distance 2 (A/B _pd2); bf16 step kernel timeline
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r5s15; mkdir -p $OUT
for v in "" _pd2; do
  XDOT_EXT_PATH=$GRAFT_REPO_ROOT/xdot/_C$v.so timeout -k 10 200 python benchmarks/bench_flash.py --dtype fp32 --fp32-mode exact --iters 5 --scores > $OUT/exact$v.log 2>&1 || exit $?
done
export XDOT_EXT_PATH=$GRAFT_REPO_ROOT/xdot/_C.so
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_bf16 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --fp32-steps 0 --no-diagnostics > $OUT/prof_bf16.log 2>&1 || exit $?
