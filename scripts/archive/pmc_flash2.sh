#!/bin/bash
# Stall anatomy of the three flash kernels at the N=1 shape: one rocprofv3 --pmc pass per
# counter group per kernel (kernel trace only, no other tracing).
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-pmc2}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for k in fwd bwd_cols bwd_rows; do
  i=0
  for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
             "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU" \
             "SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_FLAT SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp -d $OUT/${k}_g$i -o pmc --output-format csv \
      -- python3 $GRAFT_REPO_ROOT/benchmarks/bench_flash.py --iters 2 --only $k --mask > $OUT/${k}_g$i.log 2>&1 || echo "$k group $i failed rc=$?" >> $OUT/errors.log
  done
done
echo pmc-ok
