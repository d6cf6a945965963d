#!/bin/bash
# Quick GPU iteration loop: flash/module GPU tests, kernel timings (N=1 and N=8 per-rank shapes),
# the headline bench at N=1 and the emulated N=8 per-rank step.  Stops at the first failure.
set -e
O=gpurun_out/quick
mkdir -p $O
timeout -k 10 600 python -m pytest tests/test_flash_gpu.py tests/test_module_gpu.py tests/test_kernels_gpu.py -x -q -m gpu > $O/tests.log 2>&1
timeout -k 10 120 python benchmarks/bench_flash.py --mask --iters 10 > $O/flash_n1.log 2>&1
timeout -k 10 120 python benchmarks/bench_flash.py --mask --iters 20 --R 3125 > $O/flash_n8.log 2>&1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench1.log 2>&1
timeout -k 10 300 python benchmarks/bench_rank.py --world 8 --steps 20 --warmup 5 > $O/rank8.log 2>&1
echo ok
# multi-rank rehearsal: 2 ranks share the GPU over gloo (host-staged), then RCCL at N=1 under torchrun
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29622 bench.py --gpus 2 --steps 3 --warmup 1 --backend gloo > $O/gloo2.log 2>&1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29623 bench.py --gpus 1 --steps 10 --warmup 3 > $O/rccl1.log 2>&1
echo ok2
