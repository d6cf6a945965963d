#!/bin/bash
# Emulated rank steps (benchmarks/bench_rank.py) at N = 2 / 4 / 8: compute only and with the
# 300 GB/s link model, bf16 wire vs fp32 gradient wire (XDOT_GRAD_FP32=1), interleaved
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r6rank}; mkdir -p $OUT
for rep in 1 2; do
  for gf in 0 1; do
    XDOT_GRAD_FP32=$gf timeout -k 10 300 python benchmarks/bench_rank.py --world 2 4 8 --steps 20 --warmup 5 --fp32-steps 0 --no-check > $OUT/compute_gf$gf.$rep.log 2>&1 || exit $?
    XDOT_GRAD_FP32=$gf timeout -k 10 300 python benchmarks/bench_rank.py --world 8 --link-gbps 300 --p2p-gbps 64 --steps 20 --warmup 5 --fp32-steps 0 --no-check > $OUT/link_gf$gf.$rep.log 2>&1 || exit $?
  done
done
echo rank-ok
