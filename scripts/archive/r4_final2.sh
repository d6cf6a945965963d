#!/bin/bash
# Round-end health pass (smoke, GPU suite, bench shapes) followed by the exact-fp32 kernel timings.
set -o pipefail
T=${1:-r4final2}
bash scripts/r4_s3b.sh $T || exit $?
bash scripts/r4_f32k.sh $T || exit $?
echo final2-ok
