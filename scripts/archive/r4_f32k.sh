#!/bin/bash
# Exact-fp32 kernel timings: flash kernels standalone + concurrent backward pair, and BASELINE
# config 4 (LeftTranspose fwd+bwd, T=12500, one rank of 8) under a kernel trace.
set -o pipefail
T=${1:-r4f32k}
O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u benchmarks/bench_flash.py --dtype fp32 --fp32-mode exact --iters 5 --concurrent > $O/flash.log 2>&1 || exit $?
timeout -k 10 200 python benchmarks/bench_ops.py --mode leftT_fb --T 12500 --emulate 8 --dtype fp32 --iters 5 > $O/c4.log 2>&1 || exit $?
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/c4prof -o prof -- python3 $GRAFT_REPO_ROOT/benchmarks/bench_ops.py --mode leftT_fb --T 12500 --emulate 8 --dtype fp32 --iters 5 > $GRAFT_REPO_ROOT/$O/c4prof.log 2>&1 || exit $?
echo f32k-ok
