#!/bin/bash
# weight-gradient kernel: both k-steps' fragment reads before the MFMAs (XDOT_WG_PF) vs HEAD
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r6wgpf}; mkdir -p $OUT
cd $GRAFT_REPO_ROOT
XDOT_EXT_PATH=xdot/_C_wgpf.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_proj_gpu.py tests/test_kernels_gpu.py -k "wgrad or weight_grad or pair" > $OUT/pytest.log 2>&1 || { tail -20 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for rep in 1 2 3; do
  timeout -k 10 120 python benchmarks/micro/wgrad_splits.py --splits 0 --pair > $OUT/base.$rep.log 2>&1 || exit $?
  XDOT_EXT_PATH=xdot/_C_wgpf.so timeout -k 10 120 python benchmarks/micro/wgrad_splits.py --splits 0 --pair > $OUT/pf.$rep.log 2>&1 || exit $?
done
echo wgpf-ok
