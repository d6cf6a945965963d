#!/bin/bash
# Local-block-first forward at N>1: tests, then emulated per-rank steps without / with the
# link model for XDOT_LOCAL_FIRST x XDOT_GATHER_CHUNKS, then a kernel trace of the N=8 rank
# with the link model (the flash kernels vs the emulated transfer on the link stream).
set -o pipefail
TAG=${1:-overlap}; LINK=${2:-300}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_segmented.py tests/test_module_gpu.py -m gpu -q --timeout 120 \
  --timeout-method thread -rf > $O/pytest.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for lf in 0 1; do for ch in 1 2; do
  for link in none $LINK; do
    extra=""; [ $link != none ] && extra="--link-gbps $link --p2p-gbps 64"
    echo "== local_first=$lf chunks=$ch link=$link" >> $O/rank.log
    XDOT_LOCAL_FIRST=$lf XDOT_GATHER_CHUNKS=$ch timeout -k 10 300 python benchmarks/bench_rank.py --world 2 4 8 \
      --steps 20 --warmup 5 $extra >> $O/rank.log 2>&1 || exit $?
  done
done; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/trace8 -o trace \
  -- python3 $GRAFT_REPO_ROOT/benchmarks/bench_rank.py --world 8 --steps 4 --warmup 2 --link-gbps $LINK --p2p-gbps 64 \
  > $GRAFT_REPO_ROOT/$O/trace8.log 2>&1 || exit $?
echo overlap-ok
