#!/bin/bash
set -o pipefail
O=gpurun_out/${1:-r3graph2}
mkdir -p $O
timeout -k 10 900 python benchmarks/graph_ab.py --world 1 2 4 8 --steps 10 --warmup 3 > $O/graph_ab.log 2>&1 || exit $?
bash scripts/r3_ipc2.sh $1 || exit $?
echo graph2-ok
