#!/bin/bash
# Round-4 session 3: rocprofv3 kernel traces of the N=1 step and the emulated N=8 rank step at
# HEAD (bf16 only), then the reference's benchmark_results sweep re-run in the default EXACT fp32
# mode (records carry fp32_mode) into gpurun_out/<tag>/refres.
set -o pipefail
T=${1:-r4s3}
O=gpurun_out/$T
mkdir -p $O
bash scripts/gpu_prof_step.sh $T/prof || exit $?
bash scripts/gpu_ref_results.sh $O/refres || exit $?
echo s3-ok
