#!/bin/bash
# Host-side cost of the eager step at the host-bound shapes: cProfile of T=5000 N=1 (two-stream and
# one-stream attention backward) and of the emulated N=8 rank.
set -o pipefail
T=${1:-r4host}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 300 python benchmarks/host_step_profile.py --world 1 --seq-len 5000 --steps 60 --top 60 > $O/t5k.log 2>&1 || exit $?
timeout -k 10 300 python benchmarks/host_step_profile.py --world 1 --seq-len 5000 --steps 60 --top 60 --one-stream > $O/t5k_one.log 2>&1 || exit $?
timeout -k 10 300 python benchmarks/host_step_profile.py --world 8 --steps 40 --top 60 > $O/r8.log 2>&1 || exit $?
echo host-ok
