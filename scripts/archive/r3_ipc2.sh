#!/bin/bash
set -o pipefail
O=gpurun_out/${1:-r3ipc2}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
XDOT_IPC=1 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/trace -o ov_%pid% \
  -- python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 \
  $GRAFT_REPO_ROOT/benchmarks/ipc_overlap.py > $GRAFT_REPO_ROOT/$O/ov.log 2>&1 || exit $?
echo ipc2-ok
