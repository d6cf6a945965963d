#!/bin/bash
# Round 5 pass 31: the reference's benchmark_results sweep re-run at HEAD (exact fp32 products on
# the xdot GEMM kernels, no library: records carry "gemm": "xdot")
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r5s31; mkdir -p $OUT
export XDOT_EXT_PATH=$GRAFT_REPO_ROOT/xdot/_C.so
rm -rf $OUT/benchmark_results
timeout -k 10 1100 bash scripts/gpu_ref_results.sh $OUT/benchmark_results > $OUT/ref.log 2>&1
rc=$?
cp gpurun_out/ref_results.log $OUT/ 2>/dev/null
exit $rc
