#!/bin/bash
# RCCL collectives under HIP-graph capture (world 1 on the one-GPU box), then bench.py --graph
# under torchrun with the nccl backend (GraphedStep with TorchDistComm).
set -o pipefail
T=${1:-r4rgraph}
O=gpurun_out/$T; mkdir -p $O
export MASTER_ADDR=127.0.0.1
timeout -k 10 200 python -m torch.distributed.run --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 scripts/rccl_graph_check.py > $O/graph_check.log 2>&1 || exit $?
timeout -k 10 300 python -m torch.distributed.run --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29534 bench.py --graph --steps 20 --warmup 5 --fp32-steps 0 --no-check > $O/bench_graph.log 2>&1 || exit $?
echo rgraph-ok
