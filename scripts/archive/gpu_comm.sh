#!/bin/bash
# New GPU checks of this session: ring-vs-flash peak memory test, the collective micro-benchmark
# as a 2-rank one-GPU rehearsal (gloo base + IPC pull kernels), and the async-ordering suite.
set -o pipefail
TAG=${1:-comm}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_async_comm_gpu.py -v -rA --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29541 benchmarks/bench_comm.py --backend gloo --iters 10 --warmup 3 > $O/bench_comm2.log 2>&1 || exit $?
echo comm-ok
