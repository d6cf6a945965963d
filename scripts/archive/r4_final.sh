#!/bin/bash
# Round-4 closing measurements: projection tests after the route change, emulated N=2 / 4 / 8
# rank steps, kernel traces of the N=1 step and the N=8 rank step (rocprofv3 --kernel-trace
# --stats only), the multi-rank rehearsals.
set -o pipefail
T=${1:-r4final}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_proj_gpu.py tests/test_rccl_gpu.py -x -q --timeout 150 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
timeout -k 10 300 python benchmarks/bench_rank.py --world 2 4 8 --steps 20 --warmup 5 --fp32-steps 0 > $O/ranks.log 2>&1 || exit $?
timeout -k 10 300 python benchmarks/bench_rank.py --world 8 --steps 20 --warmup 5 --fp32-steps 0 --link-gbps 300 > $O/rank8_link.log 2>&1 || exit $?
bash scripts/gpu_prof_step.sh $T/prof || exit $?
bash scripts/gpu_multirank.sh $T/mr || exit $?
echo final-ok
