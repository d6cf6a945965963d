#!/bin/bash
# Same-box A/B of XDOT_RING_OVERLAP (ring backward on one vs two streams): emulated per-rank
# ring step at N=1 and N=8, 3 alternating rounds.
O=gpurun_out/ringab
mkdir -p $O
rm -f $O/*.log
for r in 1 2 3; do
  for v in 0 1; do
    XDOT_RING_OVERLAP=$v timeout -k 10 200 python benchmarks/bench_rank.py --world 1 8 --steps 20 --warmup 5 --impl ring >> $O/ov$v.log 2>&1 || exit 1
  done
done
for v in 0 1; do echo "overlap=$v: $(grep -o '"n_gpus": [0-9]*\|"value": [0-9.]*' $O/ov$v.log | paste - - | awk '{print $4"@"$2}' | tr '\n' ' ')"; done
