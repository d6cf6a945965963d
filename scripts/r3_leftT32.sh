#!/bin/bash
# fp32 LeftTransposeMultiplication fwd+bwd at the 8-rank T=12500 shape (BASELINE config 4):
# default route vs the library route vs exact fp32, and the default route's kernels.
set -o pipefail
O=gpurun_out/leftT32
mkdir -p $O
C="benchmarks/bench_ops.py --mode leftT_fb --T 12500 --emulate 8 --dtype fp32 --iters 10"
timeout -k 10 200 python $C > $O/default.log 2>&1 || exit 1
XDOT_GEMM_LIB=1 timeout -k 10 200 python $C > $O/lib.log 2>&1 || exit 1
XDOT_FP32_MODE=exact timeout -k 10 200 python $C > $O/exact.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o prof \
  -- python3 $GRAFT_REPO_ROOT/$C > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || exit 1
echo leftT32-ok
