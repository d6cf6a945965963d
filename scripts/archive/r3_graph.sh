#!/bin/bash
set -o pipefail
O=gpurun_out/${1:-r3graph}
mkdir -p $O
timeout -k 10 600 python benchmarks/graph_ab.py --world 1 8 --steps 10 --warmup 3 > $O/graph_ab.log 2>&1 || exit $?
bash scripts/r3_ipc2.sh $1 || exit $?
echo graph-ok
