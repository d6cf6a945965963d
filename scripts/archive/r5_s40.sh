#!/bin/bash
# Round 5 pass 40: per-pass kernel times of the wide column side (D = 256 h = 3, D = 384 h = 2)
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r5s40; mkdir -p $OUT
R=$GRAFT_REPO_ROOT
export XDOT_EXT_PATH=$R/xdot/_C.so
cd /tmp && export TMPDIR=/tmp
for cfg in "256 3" "384 2"; do
  set -- $cfg
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_D$1 -o run -- python3 $R/benchmarks/bench_flash.py --iters 10 --only bwd_cols --D $1 --H $2 > $OUT/cols_D$1.log 2>&1 || exit $?
done
