#!/bin/bash
# xGMI pull collectives (csrc/ipc.hip) on one MI355X: GPU tests (2-3 processes share the card),
# the headline bench as 2 ranks on the one GPU with XDOT_IPC=1 over gloo (device-side
# all-gather / reduce-scatter), and the weight-gradient GEMM sweep (xdot split-K vs hipBLASLt).
set -o pipefail
TAG=${1:-ipc}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_ipc_gpu.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
XDOT_IPC=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --backend gloo --steps 5 --warmup 2 > $O/bench2_ipc.log 2>&1 || exit $?
timeout -k 10 300 python benchmarks/bench_wgrad.py > $O/wgrad.log 2>&1 || exit $?
echo ipc-ok
