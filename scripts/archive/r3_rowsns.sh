#!/bin/bash
# rows-kernel column splits at N=1 / emulated ranks (temporary A/B knob XDOT_AB_ROWS_NS)
set -o pipefail
O=gpurun_out/${1:-r3rowsns}
mkdir -p $O
for r in 1 2; do
  for ns in 0 1 2 3 4; do
    XDOT_AB_ROWS_NS=$ns timeout -k 10 200 python bench.py --steps 20 --warmup 5 --fp32-steps 0 --no-check > $O/n1_$ns.$r.log 2>&1 || exit $?
    XDOT_AB_ROWS_NS=$ns timeout -k 10 200 python benchmarks/bench_rank.py --world 2 4 --steps 20 --warmup 5 --fp32-steps 0 --no-check > $O/nr_$ns.$r.log 2>&1 || exit $?
  done
done
echo rowsns-ok
