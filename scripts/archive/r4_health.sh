#!/bin/bash
# Round-4 health pass: smoke, full GPU suite, headline bench N=1, flash kernels standalone
# (N=1 and N=8-rank shapes, cols||rows concurrent), emulated per-rank steps.  Each GPU step has
# its own time limit; a failing step ends the script.
set -o pipefail
TAG=${1:-r4health}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke-ok')" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -rf > $O/pytest.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --fp32-steps 0 --no-check >> $O/bench.log 2>&1 || exit $?
timeout -k 10 300 python benchmarks/bench_flash.py --concurrent > $O/flash.log 2>&1 || exit $?
timeout -k 10 300 python benchmarks/bench_flash.py --R 3125 --concurrent > $O/flash8.log 2>&1 || exit $?
timeout -k 10 300 python benchmarks/bench_rank.py --world 8 --steps 20 --warmup 5 > $O/rank.log 2>&1 || exit $?
timeout -k 10 300 python benchmarks/host_step_profile.py --world 8 --steps 40 > $O/host8.log 2>&1 || exit $?
echo health-ok
