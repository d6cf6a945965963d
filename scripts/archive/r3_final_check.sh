#!/bin/bash
# Full GPU suite, smoke, the headline bench and the materialised fp32 step (split-route change).
set -o pipefail
O=gpurun_out/final
mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke-ok')" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -rf > $O/pytest.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --impl materialized --dtype fp32 --steps 3 --warmup 1 --fp32-steps 0 > $O/bench_mat_fp32.log 2>&1 || exit $?
echo final-ok
