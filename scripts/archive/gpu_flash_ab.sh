#!/bin/bash
# flash kernel env A/B: isolated + concurrent timings for each setting given as args (e.g. XDOT_COLS_NBUF=2)
set -e
O=gpurun_out/flash_ab
mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_flash_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu > $O/tests.log 2>&1
for kv in "BASE=1" "$@"; do
  env $kv timeout -k 10 200 python benchmarks/bench_flash.py --mask --iters 10 --concurrent > $O/n1_$kv.log 2>&1
  env $kv timeout -k 10 200 python benchmarks/bench_flash.py --mask --iters 10 --R 3125 --concurrent > $O/n8_$kv.log 2>&1
  env $kv XDOT_COLS_NBUF=$([ "$kv" = "XDOT_COLS_NBUF=2" ] && echo 2 || echo 3) timeout -k 10 200 python -u -m pytest tests/test_flash_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu > $O/tests_$kv.log 2>&1
done
echo ab-ok
