#!/bin/bash
# Step-level A/B of several checked-out trees (git worktrees under abtest/, each with its
# own in-tree build) plus the working tree, alternating runs of bench.py.
O=$GRAFT_REPO_ROOT/gpurun_out/cab
mkdir -p $O; rm -f $O/*.log
for r in 1 2 3; do
  for w in "$@"; do
    d=$GRAFT_REPO_ROOT; [ "$w" != "HEAD" ] && d=$GRAFT_REPO_ROOT/abtest/$w
    (cd $d && timeout -k 10 200 python bench.py --steps 20 --warmup 5 >> $O/$w.log 2>&1) || exit 1
  done
done
echo ok
