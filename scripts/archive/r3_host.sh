#!/bin/bash
# host-side profile of the emulated N=8 rank step (cProfile) + the ring path re-measured
set -o pipefail
O=gpurun_out/${1:-r3host}
mkdir -p $O
timeout -k 10 300 python -m cProfile -o $O/n8.prof benchmarks/bench_rank.py --world 8 --steps 30 --warmup 5 --fp32-steps 0 --no-check > $O/n8.log 2>&1 || exit $?
timeout -k 10 300 python benchmarks/bench_rank.py --world 2 4 8 --steps 20 --warmup 5 --fp32-steps 0 --no-check --impl ring > $O/ring.log 2>&1 || exit $?
timeout -k 10 300 python benchmarks/bench_rank.py --world 2 4 8 --steps 20 --warmup 5 --fp32-steps 0 --no-check --impl ring --link-gbps 300 --p2p-gbps 64 > $O/ring_link.log 2>&1 || exit $?
echo host-ok
