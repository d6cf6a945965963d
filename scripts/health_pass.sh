#!/bin/bash
# Health pass at HEAD: full GPU suite, smoke, default bench (bf16 + exact / split fp32
# fields), masked / unmasked ratio (interleaved), BASELINE config 1 on gloo
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r6final}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest exit $rc" >> $OUT/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.log 2>&1 || exit $?
for rep in 1 2; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --fp32-steps 0 --no-check > $OUT/mask_zeros.$rep.log 2>&1 || exit $?
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --fp32-steps 0 --no-check --mask random > $OUT/mask_random.$rep.log 2>&1 || exit $?
done
timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29631 \
  benchmarks/bench_ops.py --mode nt --T 256 --dim 64 --offset 32 --iters 5 --warmup 1 --device cpu > $OUT/c1_nt_gloo2.log 2>&1 || exit $?
echo final-ok
