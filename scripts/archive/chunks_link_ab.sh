#!/bin/bash
# A/B of XDOT_GATHER_CHUNKS 1 vs 2 on the emulated N=4 / N=8 rank step, with and without the
# 300 GB/s collective link model (3 alternating rounds).
set -o pipefail
O=gpurun_out/${1:-chunkslink}
mkdir -p $O
for r in 1 2 3; do
  for c in 1 2; do
    XDOT_GATHER_CHUNKS=$c timeout -k 10 300 python benchmarks/bench_rank.py --world 4 8 --steps 20 --warmup 5 >> $O/step_c$c.log 2>&1 || exit $?
    XDOT_GATHER_CHUNKS=$c timeout -k 10 300 python benchmarks/bench_rank.py --world 4 8 --steps 20 --warmup 5 --link-gbps 300 --p2p-gbps 64 >> $O/link_c$c.log 2>&1 || exit $?
  done
done
echo chunks-ok
