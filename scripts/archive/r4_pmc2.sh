#!/bin/bash
# PMC tables for the exact-fp32 flash kernels and the projection / weight-gradient kernels.
# Tables are built on the box and the raw per-dispatch CSVs deleted (they exceed the copy-back cap).
set -o pipefail
T=${1:-r4pmc2}
O=gpurun_out/$T
FLASH_ARGS="--dtype fp32 --fp32-mode exact" PMC_ARGS="--iters 2" bash scripts/pmc_head.sh $T/f32 || exit $?
python scripts/pmc_head_table.py $O/f32 fa32:: > $O/f32_table.md || exit $?
rm -rf $O/f32/g*/
PMC_SCRIPT=benchmarks/micro/linear_host.py PMC_ARGS="--calls 5" bash scripts/pmc_head.sh $T/lin || exit $?
python scripts/pmc_head_table.py $O/lin gemm_proj,gemm_wgrad,Cijk > $O/lin_table.md || exit $?
rm -rf $O/lin/g*/
echo pmc2-ok
