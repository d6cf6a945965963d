#!/bin/bash
# Cost side of the chunked all-gather pipeline: emulated per-rank steps (no transport) at N=2/4/8
# with XDOT_GATHER_CHUNKS=1 vs 2, alternating.
set -o pipefail
O=gpurun_out/chunks
mkdir -p $O
rm -f $O/*.log
for r in 1 2; do
  for c in 1 2; do
    XDOT_GATHER_CHUNKS=$c timeout -k 10 300 python benchmarks/bench_rank.py --world 2 4 8 --steps 20 --warmup 5 >> $O/c$c.log 2>&1 || exit 1
  done
done
for c in 1 2; do echo "chunks=$c: $(grep -o '"value": [0-9.]*\|"n_gpus": [0-9]' $O/c$c.log | paste - - | tr '\n' ' ')"; done
