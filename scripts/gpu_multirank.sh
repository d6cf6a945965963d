#!/bin/bash
# Multi-rank rehearsals on ONE GPU: 2-4 ranks over gloo (host-staged collectives, ranks share
# the card) through bench.py's own N-rank launch (no launcher in the environment: it starts
# torchrun itself) and under an explicit torchrun, flash (one-node fused module) and the
# bidirectional ring at 3 ranks; then RCCL at world size 1 under torchrun.
set -o pipefail
O=gpurun_out/${1:-multirank}
mkdir -p $O
timeout -k 10 300 python bench.py --gpus 2 --steps 3 --warmup 1 --backend gloo --fp32-steps 0 > $O/gloo2_self.log 2>&1 || exit $?
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29624 bench.py --gpus 4 --steps 3 --warmup 1 --backend gloo --fp32-steps 0 > $O/gloo4.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --gpus 3 --steps 3 --warmup 1 --backend gloo --impl ring --seq-len 24999 --fp32-steps 0 > $O/gloo3_ring.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --gpus 2 --steps 3 --warmup 1 --backend gloo --mask random --fp32-steps 0 > $O/gloo2_mask.log 2>&1 || exit $?
XDOT_FUSED_MODULE=0 timeout -k 10 300 python bench.py --gpus 2 --steps 3 --warmup 1 --backend gloo --fp32-steps 0 > $O/gloo2_nofuse.log 2>&1 || exit $?
XDOT_GATHER_CHUNKS=2 timeout -k 10 300 python bench.py --gpus 2 --steps 3 --warmup 1 --backend gloo --fp32-steps 0 > $O/gloo2_chunks2.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --gpus 2 --steps 2 --warmup 1 --backend gloo --dtype fp32 > $O/gloo2_fp32.log 2>&1 || exit $?
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29623 bench.py --gpus 1 --steps 10 --warmup 3 > $O/rccl1.log 2>&1 || exit $?
echo mr-ok
