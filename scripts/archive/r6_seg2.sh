#!/bin/bash
# kernel traces of the emulated N=8 rank step with and without the two-stream segmented forward
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r6seg2}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for s in 1 0 1 0; do
  XDOT_FWD_SEG_STREAMS=$s timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/s$s -o prof \
    -- python3 $GRAFT_REPO_ROOT/benchmarks/bench_rank.py --world 8 --steps 20 --warmup 5 --fp32-steps 0 --no-check > $OUT/s$s.log 2>&1 || exit $?
  mv $OUT/s$s $OUT/s$s.$RANDOM
done
echo seg2-ok
