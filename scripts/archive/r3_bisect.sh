#!/bin/bash
# bisect the fp16 non-finite d cols failure: batched LDS-DMA asm vs per-piece asm
set -o pipefail
O=gpurun_out/${1:-r3bisect}
mkdir -p $O
for v in nobatch batch; do
  XDOT_EXT_PATH=xdot/_C_$v.so timeout -k 10 300 python -u -m pytest tests/test_flash_gpu.py -q -m gpu --timeout 120 --timeout-method thread > $O/tests_$v.log 2>&1
  echo "$v exit $?" >> $O/summary.log
done
echo bisect-done
