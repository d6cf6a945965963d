#!/bin/bash
# PMC counters of gemm3 vs the library GEMM (hipBLASLt) on bench_gemm cases: one rocprofv3 pass
# per counter group (<= 8 SQ, <= 4 TCC, <= 2 GRBM per pass); a failing pass ends the script.
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-pmcg3}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $grp -d $OUT/g$i -o pmc --output-format csv \
    -- python3 $GRAFT_REPO_ROOT/benchmarks/bench_gemm.py --iters 3 --warmup 1 --path v3 --cases ${CASES:-ntk3072,nt_small} > $OUT/g$i.log 2>&1 || { echo "group $i failed rc=$?" >> $OUT/errors.log; exit 1; }
done
echo pmc-ok
