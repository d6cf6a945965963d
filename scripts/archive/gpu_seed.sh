#!/bin/bash
# Loss-seed change: GPU loss tests, smoke(), headline bench N=1, and a kernel-stats profile of the
# emulated N=8 rank step (the seed fill and the loss-gradient scaling kernel must be gone).
set -o pipefail
O=gpurun_out/${1:-seed}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_loss.py tests/test_split_step.py -q -m gpu --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof8 -o prof \
  -- python3 $GRAFT_REPO_ROOT/benchmarks/bench_rank.py --world 8 --steps 6 --warmup 3 > $GRAFT_REPO_ROOT/$O/prof8.log 2>&1 || exit $?
echo seed-ok
