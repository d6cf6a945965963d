#!/bin/bash
# The reference's benchmark_results/*.json sweep re-run in its own record schema
# (benchmarks/bench_ops.py --file): fp32, T = 75000 / scale, D = 768, 3 ranks — emulated on the
# one GPU (each record = ONE rank's work, collectives as device copies), plus the reference's
# single-GPU torch.matmul baseline on the full problem; collectives priced by the link model
# (EmulatedComm link_gbps, default 300 GB/s all-gather bus bandwidth per rank; LINK_GBPS=).
# 101 records per file: the summary
# record, then 100 trials (one synchronised call each), as the reference's 100-trial files.
set -o pipefail
O=${1:-benchmark_results}
mkdir -p $O gpurun_out
run() {  # file, args...
  f=$1; shift
  timeout -k 10 120 python benchmarks/bench_ops.py --emulate 3 --link-gbps ${LINK_GBPS:-300} --iters 3 --warmup 1 --trials 101 --file $O/$f "$@" \
    >> gpurun_out/ref_results.log 2>&1 || { echo "failed: $f $*" >> gpurun_out/ref_results.log; return 1; }
}
for o in 1000 1250 2500 5000 6250 12500 25000; do run nt_benchmark_$o.json --mode nt --offset $o || exit 1; done
run nt_benchmark.json --mode nt || exit 1
for s in 1 2 4 8; do run nt_benchmark_size_$s.json --mode nt --offset 1000 --scale $s || exit 1; done
for o in 2 24 48 96 192 384 768; do run all_benchmark_$o.json --mode all --offset $o || exit 1; done
for s in 1 2 4 8; do run all_benchmark_size_$s.json --mode all --offset 1000 --scale $s || exit 1; done
for s in 1 2 4 8; do run tn_benchmark_$s.json --mode tn --scale $s || exit 1; done
echo ref-results-ok
