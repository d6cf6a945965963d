#!/bin/bash
# A/B: optimizer step split around the last gradient all-reduce (default) vs one step after the
# wait (--no-split-step), emulated N=4 / N=8 rank with and without the 300 GB/s link model.
set -o pipefail
O=gpurun_out/${1:-splitstep}
mkdir -p $O
for r in 1 2 3; do
  for arm in A B; do
    x=$([ $arm == A ] && echo "--no-split-step" || echo "")
    timeout -k 10 300 python benchmarks/bench_rank.py --world 4 8 --steps 30 --warmup 5 $x >> $O/step_$arm.log 2>&1 || exit $?
    timeout -k 10 300 python benchmarks/bench_rank.py --world 4 8 --steps 30 --warmup 5 --link-gbps 300 --p2p-gbps 64 $x >> $O/link_$arm.log 2>&1 || exit $?
  done
done
echo split-ok
