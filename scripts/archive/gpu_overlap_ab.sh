#!/bin/bash
# Alternating A/B of the multi-rank schedule knobs at emulated N=8 (and 4), without and with
# the link model: 3 rounds x {XDOT_LOCAL_FIRST, XDOT_GATHER_CHUNKS} configs.
set -o pipefail
TAG=${1:-ovab}; LINK=${2:-300}; WORLDS=${3:-"4 8"}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_segmented.py tests/test_module_gpu.py -m gpu -q --timeout 120 \
  --timeout-method thread -rf > $O/pytest.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for round in 1 2 3; do
  for cfg in "0 1" "1 1" "1 2" "1 3"; do
    set -- $cfg
    for link in none $LINK; do
      extra=""; [ $link != none ] && extra="--link-gbps $link --p2p-gbps 64"
      echo "== round=$round local_first=$1 chunks=$2 link=$link" >> $O/rank.log
      XDOT_LOCAL_FIRST=$1 XDOT_GATHER_CHUNKS=$2 timeout -k 10 300 python benchmarks/bench_rank.py --world $WORLDS \
        --steps 30 --warmup 5 $extra >> $O/rank.log 2>&1 || exit $?
    done
  done
done
echo ab-ok
