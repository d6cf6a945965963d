#!/bin/bash
# Projection kernel variants (xdot/_C_<v>.so from scripts/build_variant.sh): correctness of the
# 3-stage ring, then hipBLASLt vs each variant per shape; the side-stream GPU test; the steps
# at the new defaults.
set -o pipefail
T=${1:-r4projab}
O=gpurun_out/$T
mkdir -p $O
for v in ns3 nobig3; do
  XDOT_EXT_PATH=xdot/_C_$v.so timeout -k 10 300 python -u -m pytest tests/test_proj_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest_$v.log 2>&1 || exit $?
done
timeout -k 10 300 python benchmarks/micro/linear_host.py > $O/lh_base_full.log 2>&1 || exit $?
for v in prio ns3 ns3p nobig3; do
  XDOT_EXT_PATH=xdot/_C_$v.so timeout -k 10 300 python benchmarks/micro/linear_host.py --quick > $O/lh_$v.log 2>&1 || exit $?
done
timeout -k 10 300 python benchmarks/micro/linear_host.py --quick > $O/lh_base2.log 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest tests/test_module_gpu.py -x -q --timeout 120 --timeout-method thread -k "side_stream or deterministic or single_rank" > $O/pytest_module.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --fp32-steps 0 --no-check > $O/n1.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --seq-len 5000 --steps 50 --warmup 10 --fp32-steps 0 --no-check > $O/t5k.log 2>&1 || exit $?
timeout -k 10 200 python benchmarks/bench_rank.py --world 8 --steps 30 --warmup 5 --fp32-steps 0 > $O/r8.log 2>&1 || exit $?
timeout -k 10 200 python benchmarks/bench_rank.py --world 8 --rank 3 --steps 30 --warmup 5 --fp32-steps 0 > $O/r8_rank3.log 2>&1 || exit $?
timeout -k 10 300 python benchmarks/host_step_profile.py --world 8 --steps 40 --inline-backward > $O/host8.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_module_gpu.py tests/test_ring_ops.py -x -q --timeout 300 --timeout-method thread -k "ring" > $O/pytest_ring.log 2>&1 || exit $?
timeout -k 10 300 python benchmarks/bench_rank.py --world 8 --steps 10 --warmup 3 --impl ring --link-gbps 300 --p2p-gbps 64 --fp32-steps 0 > $O/ring8.log 2>&1 || exit $?
XDOT_RING_BIDIR=0 timeout -k 10 300 python benchmarks/bench_rank.py --world 8 --steps 10 --warmup 3 --impl ring --link-gbps 300 --p2p-gbps 64 --fp32-steps 0 > $O/ring8_uni.log 2>&1 || exit $?
echo projab-ok
