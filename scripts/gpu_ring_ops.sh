#!/bin/bash
# Ring schedule of the distributed products: GPU numerics (3 gloo ranks) and emulated N=8 timings
# of config 3 (T=25000, nt / all) and tn, gather vs ring, without and with the link model
# (collectives 300 GB/s, ring hops 64 GB/s).  Records: gpurun_out/<tag>/
set -o pipefail
O=gpurun_out/${1:-ring_ops}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gemm2_gpu.py tests/test_ops_gpu.py -q -m gpu --timeout 300 --timeout-method thread -x > $O/tests.log 2>&1 || exit $?
echo tests-ok
for m in nt all tn; do
  for s in gather ring; do
    timeout -k 10 200 python benchmarks/bench_ops.py --mode $m --T 25000 --emulate 8 --dtype bf16 --iters 5 --schedule $s --no-local > $O/${m}_$s.log 2>&1 || exit $?
    timeout -k 10 200 python benchmarks/bench_ops.py --mode $m --T 25000 --emulate 8 --dtype bf16 --iters 5 --schedule $s --no-local \
      --link-gbps 300 --p2p-gbps 64 > $O/${m}_${s}_link.log 2>&1 || exit $?
  done
done
echo bench-ok
