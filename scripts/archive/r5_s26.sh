#!/bin/bash
# Round 5 pass 26: full GPU suite + smoke + default bench at HEAD (health)
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r5s26; mkdir -p $OUT
export XDOT_EXT_PATH=$GRAFT_REPO_ROOT/xdot/_C.so
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest exit $rc" >> $OUT/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > $OUT/bench.log 2>&1 || exit $?
