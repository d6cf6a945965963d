#!/bin/bash
# Fill-aware split-fp32 cost model: fp32 configs 3/4 of BASELINE.json per rank of 8, library and
# exact routes for comparison, then the GEMM / op / fp32 GPU tests.
set -o pipefail
O=gpurun_out/fillm
mkdir -p $O
for m in "leftT_fb --T 12500" "nt --T 25000 --offset 32" "all --T 25000 --offset 32" "rightT_fb --T 12500" "full_fb --T 12500"; do
  for env in "" "XDOT_GEMM_LIB=1" "XDOT_FP32_MODE=exact"; do
    r=$(env $env timeout -k 10 200 python benchmarks/bench_ops.py --mode $m --emulate 8 --dtype fp32 --iters 10 2>/dev/null | grep '"mode"') || exit 1
    echo "$m [$env] $(echo "$r" | python -c 'import sys,json;print(json.loads(sys.stdin.read())["ms_p50"])')" >> $O/ops.log
  done
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "gemm or ops or mult or f32 or fp32 or module or gradient" > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; cat $O/ops.log; exit $rc
