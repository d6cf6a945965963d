#!/bin/bash
# weight-gradient route A/B: gemm3 (path 5, default) vs the v2 kernel (path 2), standalone and in
# the headline step (N=1) and the emulated N=8 rank step; 2 alternating rounds.
set -o pipefail
O=gpurun_out/wgrad_ab
mkdir -p $O
for p in 5 2; do
  timeout -k 10 300 python -c "import sys; sys.argv=['bench_wgrad']; import xdot.ops.linear as L; L._WGRAD_PATH=$p; import runpy; runpy.run_path('benchmarks/bench_wgrad.py', run_name='__main__')" > $O/wgrad_p$p.log 2>&1 || exit 1
done
for r in 1 2; do
  for p in 5 2; do
    timeout -k 10 300 python -c "import sys; sys.argv=['bench.py','--steps','20','--warmup','5']; import xdot.ops.linear as L; L._WGRAD_PATH=$p; import runpy; runpy.run_path('bench.py', run_name='__main__')" > $O/step_p${p}_r$r.log 2>&1 || exit 1
    timeout -k 10 300 python -c "import sys; sys.argv=['bench_rank','--world','8']; import xdot.ops.linear as L; L._WGRAD_PATH=$p; import runpy; runpy.run_path('benchmarks/bench_rank.py', run_name='__main__')" > $O/rank8_p${p}_r$r.log 2>&1 || exit 1
  done
done
for f in $O/wgrad_p*.log; do echo $f; cat $f; done
for f in $O/step_p*.log; do echo $f $(tail -1 $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'])"); done
for f in $O/rank8_p*.log; do echo $f; tail -2 $f; done
