#!/bin/bash
# Reference per-op benchmark configs (benchmark_results/*.json: fp32, D=768, T=75000/scale, N=3)
# on one MI355X: N=3 per-rank work via --emulate 3 (collectives are device-local copies) and
# the whole problem on one GPU (N=1).  Records go to gpurun_out/ops/ops.json.
# Usage (via gpurun): bash scripts/archive/gpu_ops.sh
set -e
O=gpurun_out/ops
mkdir -p $O
J=$O/ops.json
run() { timeout -k 10 240 python benchmarks/bench_ops.py --iters 5 --warmup 2 --file $J "$@" >> $O/ops.log 2>&1; }
run --mode nt --offset 1000 --emulate 3
run --mode nt --emulate 3
run --mode nt --offset 25000 --emulate 3
run --mode all --emulate 3
run --mode all --offset 24 --emulate 3
run --mode tn --emulate 3
for s in 2 4 8; do
  run --mode nt --scale $s --emulate 3
  run --mode all --scale $s --emulate 3
  run --mode tn --scale $s --emulate 3
done
run --mode nt
run --mode all
run --mode tn
run --mode nt --dtype bf16
run --mode all --dtype bf16
run --mode tn --dtype bf16
run --mode rightT_fb --emulate 3
run --mode full_fb --emulate 3
run --mode leftT_fb --emulate 3
echo ops-ok
timeout -k 10 300 python benchmarks/bench_rank.py --world 2 4 8 --steps 20 --warmup 5 > $O/rank.log 2>&1
echo rank-ok
