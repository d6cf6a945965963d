#!/bin/bash
# The xGMI pull collectives at world size 4 and 8 (all ranks on the one GPU of this box, gloo for
# the handle exchange and the parameter all-reduce): headline bench over IPC, and the collective
# micro-benchmark at 8 ranks.
set -o pipefail
O=gpurun_out/${1:-ipc8}
mkdir -p $O
for n in 4 8; do
  XDOT_IPC=1 XDOT_IPC_MB=128 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port 2955$n bench.py --gpus $n --backend gloo --steps 5 --warmup 2 > $O/bench_ipc$n.log 2>&1 || exit $?
done
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
  --master-port 29561 benchmarks/bench_comm.py --backend gloo --iters 5 --warmup 2 > $O/bench_comm8.log 2>&1 || exit $?
echo ipc8-ok
