#!/bin/bash
# IPC overlap evidence: the 2-process same-GPU rehearsal (gloo for the host exchange, XDOT_IPC=1
# device pull collectives) of the headline step at T=25000 (R=12500 per rank), under a kernel
# trace; then the IPC tests (async handle / NaN poisoning / module step).
set -o pipefail
O=gpurun_out/${1:-r3ipc}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_ipc_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
XDOT_IPC=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/trace -o ipc \
  -- python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  $GRAFT_REPO_ROOT/bench.py --gpus 2 --backend gloo --steps 4 --warmup 2 --fp32-steps 0 --no-check > $GRAFT_REPO_ROOT/$O/bench.log 2>&1 || exit $?
echo ipc-ok
