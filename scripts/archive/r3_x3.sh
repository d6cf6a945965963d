#!/bin/bash
# split-bf16 fp32 mode: GPU tests, then the exact-vs-split A/B (errors, kernels, step)
set -o pipefail
O=gpurun_out/${1:-r3x3}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_flash_f32_gpu.py > $O/tests.log 2>&1 || exit $?
timeout -k 10 400 python -u benchmarks/fp32_split_ab.py --iters 5 --steps 5 > $O/ab.log 2>&1 || exit $?
bash scripts/r3_ipc2.sh $1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/rank8 -o prof \
  -- python3 $GRAFT_REPO_ROOT/benchmarks/bench_rank.py --world 8 --steps 10 --warmup 3 --fp32-steps 0 --no-check > $GRAFT_REPO_ROOT/$O/rank8.log 2>&1 || exit $?
echo x3-ok
