#!/bin/bash
# Round 5 pass 12: PMC of the 256x256 fp32 GEMM (nt / tn shapes) and of the fp32 score-buffer
# kernels after the select-free softmax; per-kernel stats of both fp32 families
set -o pipefail
export XDOT_EXT_PATH=$GRAFT_REPO_ROOT/xdot/_C.so
OUT=$GRAFT_REPO_ROOT/gpurun_out/r5s12; mkdir -p $OUT
PMC_SCRIPT=benchmarks/bench_gemm.py PMC_ARGS="--dtype fp32 --path v2 --cases nt_wide,tn3 --iters 2 --warmup 1" bash scripts/pmc_head.sh r5s12/pmc_gemm2f32 || exit $?
FLASH_ARGS="--dtype fp32 --fp32-mode exact --scores" bash scripts/pmc_head.sh r5s12/pmc_f32sb || exit $?
cd /tmp && export TMPDIR=/tmp
for m in exact split; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$m -o run -- python3 $GRAFT_REPO_ROOT/benchmarks/bench_flash.py --dtype fp32 --fp32-mode $m --iters 3 --scores > $OUT/prof_$m.log 2>&1 || exit $?
done
