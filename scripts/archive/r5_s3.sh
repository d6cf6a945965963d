#!/bin/bash
# Round 5 pass 3: the exact-fp32 GEMM (gemm_f32.hip) vs the library, its tests, then pass 2's list.
set -o pipefail
OUT=gpurun_out/r5s3; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gemm_f32_gpu.py > $OUT/pytest_gemm.log 2>&1
rc=$?; echo "pytest exit $rc" >> $OUT/pytest_gemm.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python benchmarks/bench_gemm.py --dtype fp32 --cases proj,proj_dx,wgrad,nt_wide,all3,tn3 --iters 5 --warmup 2 > $OUT/gemm_f32.log 2>&1 || exit $?
bash scripts/r5_s2.sh
