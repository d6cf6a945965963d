#!/bin/bash
# gather chunks at the emulated N=8 rank (XDOT_GATHER_CHUNKS 1 / 2 / 3), link model and compute only, interleaved
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r6chunks}; mkdir -p $OUT
cd $GRAFT_REPO_ROOT
for rep in 1 2; do
  for c in 1 2 3; do
    XDOT_GATHER_CHUNKS=$c timeout -k 10 300 python benchmarks/bench_rank.py --world 8 --link-gbps 300 --p2p-gbps 64 --steps 20 --warmup 5 --fp32-steps 0 --no-check > $OUT/link_c$c.$rep.log 2>&1 || exit $?
    XDOT_GATHER_CHUNKS=$c timeout -k 10 300 python benchmarks/bench_rank.py --world 8 --steps 20 --warmup 5 --fp32-steps 0 --no-check > $OUT/comp_c$c.$rep.log 2>&1 || exit $?
    echo "c$c rep$rep link $(grep -o '"ms_per_step": [0-9.]*' $OUT/link_c$c.$rep.log) comp $(grep -o '"ms_per_step": [0-9.]*' $OUT/comp_c$c.$rep.log)"
  done
done
