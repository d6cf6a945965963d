#!/bin/bash
# Row-kernel column splits at the N=8 per-rank shape (R=3125, T=25000): standalone kernels and
# cols||rows on two streams, per nsplit (0 = automatic choice).
set -o pipefail
O=gpurun_out/splits
mkdir -p $O
rm -f $O/*.log
for ns in 0 2 3 4 6 8; do
  timeout -k 10 120 python benchmarks/bench_flash.py --R 3125 --T 25000 --nsplit $ns --concurrent --iters 20 --only bwd_rows >> $O/ns_$ns.log 2>&1 || exit 1
done
for ns in 0 2 3 4 6 8; do echo "nsplit=$ns: $(grep -o '"kernel": "[^"]*", "ms": [0-9.]*' $O/ns_$ns.log | tr '\n' ' ')"; done
