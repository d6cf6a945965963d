#!/bin/bash
# Round 6 health pass: full GPU suite, smoke, default bench (bf16 + exact / split fp32 fields)
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r6h}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest exit $rc" >> $OUT/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > $OUT/bench.log 2>&1 || exit $?
if [ -n "$R6_EXTRA" ]; then eval "$R6_EXTRA" || exit $?; fi
