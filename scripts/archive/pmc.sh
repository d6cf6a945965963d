#!/bin/bash
# Collect PMC counter groups for a command, one rocprofv3 pass per group (no tracing domains).
#   bash scripts/archive/pmc.sh <out-tag> "<grp1 counters>" "<grp2 counters>" ... -- <python args...>
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/$1; shift
groups=()
while [ "$1" != "--" ] && [ $# -gt 0 ]; do groups+=("$1"); shift; done
shift
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "${groups[@]}"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $grp -d $OUT/g$i -o pmc --output-format csv \
    -- python3 $GRAFT_REPO_ROOT/"$@" > $OUT/g$i.log 2>&1 || { echo "group $i failed rc=$?" >> $OUT/errors.log; exit 1; }
done
