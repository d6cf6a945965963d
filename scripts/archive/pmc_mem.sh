#!/bin/bash
# Memory-side PMC counters of the flash kernels (one rocprofv3 pass per group, no tracing).
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-pmcmem}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE" \
           "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum" \
           "SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_INSTS_VALU_TRANS_F SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INST_LEVEL_LDS"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $grp -d $OUT/g$i -o pmc --output-format csv \
    -- python3 $GRAFT_REPO_ROOT/benchmarks/bench_flash.py --iters 3 > $OUT/g$i.log 2>&1 || { echo "group $i failed rc=$?" >> $OUT/errors.log; exit 1; }
done
