#!/bin/bash
# PMC tables for the exact-fp32 flash kernels and the projection / weight-gradient kernels.
set -o pipefail
T=${1:-r4pmc2}
FLASH_ARGS="--dtype fp32 --fp32-mode exact" bash scripts/pmc_head.sh $T/f32 || exit $?
PMC_SCRIPT=benchmarks/micro/linear_host.py PMC_ARGS="--calls 20" bash scripts/pmc_head.sh $T/lin || exit $?
echo pmc2-ok
