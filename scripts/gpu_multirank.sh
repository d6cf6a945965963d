#!/bin/bash
# Multi-rank rehearsals on ONE GPU: 2 and 4 ranks over gloo (host-staged collectives, ranks
# share the card), then RCCL at world size 1 under torchrun.  Correctness of the N>1 paths.
set -e
O=gpurun_out/${1:-multirank}
mkdir -p $O
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29622 bench.py --gpus 2 --steps 3 --warmup 1 --backend gloo > $O/gloo2.log 2>&1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29624 bench.py --gpus 4 --steps 3 --warmup 1 --backend gloo > $O/gloo4.log 2>&1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29625 bench.py --gpus 2 --steps 3 --warmup 1 --backend gloo --mask random > $O/gloo2_mask.log 2>&1
XDOT_GATHER_CHUNKS=2 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29626 bench.py --gpus 2 --steps 3 --warmup 1 --backend gloo > $O/gloo2_chunks2.log 2>&1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29627 bench.py --gpus 2 --steps 3 --warmup 1 --backend gloo --dtype fp32 > $O/gloo2_fp32.log 2>&1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29623 bench.py --gpus 1 --steps 10 --warmup 3 > $O/rccl1.log 2>&1
echo mr-ok
