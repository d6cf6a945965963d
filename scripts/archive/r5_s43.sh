#!/bin/bash
# Round 5 pass 43: r5s42's remaining arms (fp32 D = 384 needs the score buffer: --scores) and a
# second repetition, then PMC of the D = 256 bf16 kernels
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r5s43; mkdir -p $OUT
R=$GRAFT_REPO_ROOT
for rep in 1 2; do
  for v in _C _C_noselb; do
    XDOT_EXT_PATH=$R/xdot/$v.so timeout -k 10 200 python benchmarks/bench_flash.py --iters 10 --D 384 --H 2 > $OUT/$v.D384.$rep.log 2>&1 || exit $?
    XDOT_EXT_PATH=$R/xdot/$v.so timeout -k 10 300 python benchmarks/bench_flash.py --iters 5 --D 256 --H 3 --dtype fp32 --fp32-mode exact > $OUT/$v.f32D256.$rep.log 2>&1 || exit $?
    XDOT_EXT_PATH=$R/xdot/$v.so timeout -k 10 300 python benchmarks/bench_flash.py --iters 5 --D 384 --H 2 --dtype fp32 --fp32-mode exact --scores > $OUT/$v.f32D384.$rep.log 2>&1 || exit $?
  done
  for v in _C _C_cocc1; do
    XDOT_EXT_PATH=$R/xdot/$v.so timeout -k 10 200 python benchmarks/bench_flash.py --iters 10 --D 256 --H 3 --only bwd_cols > $OUT/$v.D256.$rep.log 2>&1 || exit $?
  done
done
