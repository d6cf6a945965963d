#!/bin/bash
# Kernel trace of the emulated N=8 rank step with the 300 GB/s collective link model (spin kernels
# on the collective stream stand for the transfers): where the modelled transport is exposed
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r6link}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/link8 -o prof \
  -- python3 $GRAFT_REPO_ROOT/benchmarks/bench_rank.py --world 8 --link-gbps 300 --p2p-gbps 64 --steps 6 --warmup 3 --fp32-steps 0 --no-check > $O/link8.log 2>&1 || exit $?
echo link-ok
