#!/bin/bash
# PMC counters of the GEMM kernels (xdot gemm2 vs hipBLASLt on the same shape), one pass per group.
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-pmc_gemm}
CASE=${2:-nt_small}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
           "SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_VALU" \
           "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" \
           "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TA_BUSY_avr TA_TA_BUSY_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $grp -d $OUT/g$i -o pmc --output-format csv \
    -- python3 $GRAFT_REPO_ROOT/benchmarks/bench_gemm.py --cases $CASE --iters 2 --warmup 1 > $OUT/g$i.log 2>&1 || echo "group $i failed rc=$?" >> $OUT/errors.log
done
echo pmc-done
