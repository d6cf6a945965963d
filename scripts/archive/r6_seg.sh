#!/bin/bash
# Two-stream segmented forward (XDOT_FWD_SEG_STREAMS) + FusedAdamW fp32-gradient write-back:
# GPU tests, emulated rank A/B (compute only and with the link model), N=8 kernel trace
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r6seg}; mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_kernels_gpu.py tests/test_module_gpu.py tests/test_async_comm_gpu.py tests/test_production_shape_gpu.py \
  tests/test_graphs_gpu.py tests/test_rccl_gpu.py tests/test_segmented.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for rep in 1 2; do
  for s in 1 0; do
    XDOT_FWD_SEG_STREAMS=$s timeout -k 10 300 python benchmarks/bench_rank.py --world 2 4 8 --steps 20 --warmup 5 --fp32-steps 0 --no-check > $OUT/compute_s$s.$rep.log 2>&1 || exit $?
    XDOT_FWD_SEG_STREAMS=$s timeout -k 10 300 python benchmarks/bench_rank.py --world 8 --link-gbps 300 --p2p-gbps 64 --steps 20 --warmup 5 --fp32-steps 0 --no-check > $OUT/link_s$s.$rep.log 2>&1 || exit $?
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/rank8 -o prof \
  -- python3 $GRAFT_REPO_ROOT/benchmarks/bench_rank.py --world 8 --steps 8 --warmup 3 --fp32-steps 0 --no-check > $OUT/rank8.log 2>&1 || exit $?
echo seg-ok
