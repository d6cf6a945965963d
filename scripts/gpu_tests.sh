#!/bin/bash
# GPU test suite only (no -x: every failure is listed), one time limit for the whole run.
# Usage: bash scripts/gpu_tests.sh <tag> [pytest selectors...]
set -o pipefail
TAG=${1:-tests}; shift
O=gpurun_out/$TAG
mkdir -p $O
SEL=${@:-tests}
timeout -k 10 900 python -u -m pytest $SEL -m gpu -q --timeout 120 --timeout-method thread -rf > $O/pytest.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/pytest.log
exit $rc
