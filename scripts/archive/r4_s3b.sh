#!/bin/bash
# Health pass after the projection routing / inline backward / side-stream default changes:
# smoke, the whole GPU suite, the default bench, the step shapes, host profile, ring.
set -o pipefail
T=${1:-r4s3b}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke-ok')" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -rf > $O/pytest.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --fp32-steps 0 --no-check >> $O/bench.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --seq-len 5000 --steps 50 --warmup 10 --fp32-steps 0 --no-check > $O/t5k.log 2>&1 || exit $?
timeout -k 10 200 python benchmarks/bench_rank.py --world 8 --steps 30 --warmup 5 --fp32-steps 0 > $O/r8.log 2>&1 || exit $?
timeout -k 10 300 python benchmarks/host_step_profile.py --world 8 --steps 40 > $O/host8.log 2>&1 || exit $?
timeout -k 10 300 python benchmarks/micro/linear_host.py --quick > $O/linear_host.log 2>&1 || exit $?
echo s3b-ok
