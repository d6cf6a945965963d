#!/bin/bash
# A/B of one environment switch: flash GPU tests under both values, per-kernel timings
# (bench_flash, N=1 shapes), the headline bench (N=1) and the emulated N=8 rank step,
# alternating A/B runs.  usage: ab_full.sh VAR valA valB [rounds]
VAR=$1; A=$2; B=$3; N=${4:-3}
O=gpurun_out/abfull
mkdir -p $O
rm -f $O/*.log
tag() { local t=${1//\//_}; echo ${t:-default}; }
for v in "$A" "$B"; do
  env $VAR=$v timeout -k 10 300 python -m pytest tests/test_flash_gpu.py tests/test_module_gpu.py tests/test_long_context_gpu.py -x -q -m gpu > $O/tests_$(tag $v).log 2>&1 || { echo "tests failed under $VAR=$v"; exit 1; }
done
for r in $(seq $N); do
  for v in "$A" "$B"; do
    env $VAR=$v timeout -k 10 120 python benchmarks/bench_flash.py >> $O/flash_$(tag $v).log 2>&1 || exit 1
    env $VAR=$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 >> $O/bench_$(tag $v).log 2>&1 || exit 1
    env $VAR=$v timeout -k 10 200 python benchmarks/bench_rank.py --world 8 --steps 30 --warmup 5 >> $O/rank8_$(tag $v).log 2>&1 || exit 1
  done
done
for v in "$A" "$B"; do
  t=$(tag $v)
  echo "$VAR=$t bench: $(grep -o '"value": [0-9.]*' $O/bench_$t.log | awk '{print $2}' | tr '\n' ' ')  rank8: $(grep -o '"value": [0-9.]*' $O/rank8_$t.log | awk '{print $2}' | tr '\n' ' ')"
done
