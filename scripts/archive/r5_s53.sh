#!/bin/bash
# Round 5 pass 53: emulated per-rank steps at the closing HEAD (compute only; N = 2 / 4 / 8) and the N = 8
# rank with collectives priced at 300 GB/s
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r5s53; mkdir -p $OUT
export XDOT_EXT_PATH=$GRAFT_REPO_ROOT/xdot/_C.so
timeout -k 10 400 python benchmarks/bench_rank.py --world 2 4 8 > $OUT/rank.log 2>&1 || exit $?
timeout -k 10 300 python benchmarks/bench_rank.py --world 8 --link-gbps 300 > $OUT/rank8_link.log 2>&1 || exit $?
