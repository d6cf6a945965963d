#!/bin/bash
# Round health pass: full GPU suite, headline bench N=1, emulated per-rank N=2/4/8 (with and
# without the 300 GB/s link model), rocprofv3 kernel stats of the N=1 step and a kernel trace of
# the emulated N=8 rank step (bf16 steps only: --fp32-steps 0, so the tables do not blend in the
# fp32 companion's kernels).  Every GPU step has its own time limit; a failing step ends it.
set -o pipefail
TAG=${1:-health}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke-ok')" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -rf > $O/pytest.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || exit $?
timeout -k 10 300 python benchmarks/bench_rank.py --world 2 4 8 --steps 20 --warmup 5 > $O/rank.log 2>&1 || exit $?
timeout -k 10 300 python benchmarks/bench_rank.py --world 2 4 8 --steps 20 --warmup 5 --link-gbps 300 --p2p-gbps 64 > $O/rank_link.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --dtype fp32 --steps 5 --warmup 2 > $O/bench_fp32.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --impl materialized --steps 5 --warmup 2 > $O/bench_mat.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --impl materialized --dtype fp32 --steps 3 --warmup 1 > $O/bench_mat_fp32.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o prof \
  -- python3 $GRAFT_REPO_ROOT/bench.py --steps 4 --warmup 2 --fp32-steps 0 --no-check > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof8 -o prof \
  -- python3 $GRAFT_REPO_ROOT/benchmarks/bench_rank.py --world 8 --steps 6 --warmup 3 --fp32-steps 0 > $GRAFT_REPO_ROOT/$O/prof8.log 2>&1 || exit $?
echo health-ok
