#!/bin/bash
# BASELINE.json's five configs, measured on one MI355X (multi-GPU configs: ONE rank's work
# emulated, collectives as device-local copies).  Records: gpurun_out/cfg/*.log
set -e
O=gpurun_out/${1:-cfg}
mkdir -p $O
# 1. distributed_matmul_nt CPU/gloo world_size=2, T=256 d=64 offset=32 (plumbing, no GPU)
timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29631 \
  benchmarks/bench_ops.py --mode nt --T 256 --dim 64 --offset 32 --iters 5 --warmup 1 --device cpu > $O/c1_nt_gloo2.log 2>&1 || echo c1-failed >> $O/c1_nt_gloo2.log
echo c1
# 2. DistributedDotProductAttn 1xMI355X, T=5000 d=768 heads=8 bf16
timeout -k 10 200 python bench.py --seq-len 5000 --steps 50 --warmup 10 > $O/c2_attn_T5000.log 2>&1
echo c2
# 3. nt + all, 8 ranks, T=25000 d=768 offset=32 (one rank emulated), bf16 and fp32
for dt in bf16 fp32; do
  timeout -k 10 200 python benchmarks/bench_ops.py --mode nt --T 25000 --offset 32 --emulate 8 --dtype $dt --iters 5 > $O/c3_nt_$dt.log 2>&1
  timeout -k 10 200 python benchmarks/bench_ops.py --mode all --T 25000 --offset 32 --emulate 8 --dtype $dt --iters 5 > $O/c3_all_$dt.log 2>&1
done
for m in nt all; do  # with the 300 GB/s collective link model
  timeout -k 10 200 python benchmarks/bench_ops.py --mode $m --T 25000 --offset 32 --emulate 8 --dtype bf16 --iters 5 \
    --link-gbps 300 > $O/c3_${m}_bf16_link300.log 2>&1
done
echo c3
# 4. LeftTransposeMultiplication fwd+bwd, 8 ranks, T=12500 (one rank emulated)
timeout -k 10 200 python benchmarks/bench_ops.py --mode leftT_fb --T 12500 --emulate 8 --dtype bf16 --iters 5 > $O/c4_leftT_bf16.log 2>&1
timeout -k 10 200 python benchmarks/bench_ops.py --mode leftT_fb --T 12500 --emulate 8 --dtype fp32 --iters 5 > $O/c4_leftT_fp32.log 2>&1
timeout -k 10 200 python benchmarks/bench_ops.py --mode leftT_fb --T 12500 --offset 32 --emulate 8 --dtype bf16 --iters 5 > $O/c4_leftT_bf16_o32.log 2>&1
echo c4
# 5. long context T=200000, d=768, h=8, 8 ranks (one rank emulated: R=25000 rows x T=200000), bf16
timeout -k 10 300 python benchmarks/bench_rank.py --world 8 --seq-len 200000 --steps 3 --warmup 1 > $O/c5_T200000_n8.log 2>&1
echo c5-ok
