#!/bin/bash
# Flash kernel diagnostics: isolated + concurrent timings vs torch SDPA, then PMC groups per kernel.
set -e
O=gpurun_out/flashdiag
mkdir -p $O
timeout -k 10 300 python benchmarks/bench_flash.py --mask --iters 10 --concurrent --torch > $O/n1.log 2>&1
timeout -k 10 300 python benchmarks/bench_flash.py --mask --iters 10 --R 3125 --concurrent > $O/n8.log 2>&1
echo timing-ok
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_VALU_MFMA_BUSY_CYCLES" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC" \
           "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp -d $GRAFT_REPO_ROOT/$O/g$i -o pmc --output-format csv \
    -- python3 $GRAFT_REPO_ROOT/benchmarks/bench_flash.py --mask --iters 2 > $GRAFT_REPO_ROOT/$O/g$i.log 2>&1 || echo "group $i failed" >> $GRAFT_REPO_ROOT/$O/errors.log
done
echo pmc-ok
