#!/bin/bash
# Round 5 pass 10: long context at the reference example's config (T = 200000, d = 768, h = 2 ->
# D = 384, N = 1, bf16 flash); GEMM auto route after the heuristic change; bf16 HEAD PMC refresh
set -o pipefail
export XDOT_EXT_PATH=$GRAFT_REPO_ROOT/xdot/_C.so
OUT=$GRAFT_REPO_ROOT/gpurun_out/r5s10; mkdir -p $OUT
timeout -k 10 300 python bench.py --seq-len 200000 --heads 2 --steps 3 --warmup 1 --fp32-steps 0 > $OUT/long_h2.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --seq-len 200000 --heads 8 --steps 3 --warmup 1 --fp32-steps 0 > $OUT/long_h8.log 2>&1 || exit $?
timeout -k 10 300 python benchmarks/bench_gemm.py --dtype fp32 --cases proj,proj_dx,wgrad,nt_wide,all3,tn3 --iters 5 > $OUT/gemm_auto.log 2>&1 || exit $?
bash scripts/pmc_head.sh r5s10/pmc_bf16 || exit $?
