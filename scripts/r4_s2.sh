#!/bin/bash
# Round-4 session 2: forward row-max A/B (tree vs chain), host profile with the backward inline,
# HEAD PMC table of the flash kernels, exact-fp32 BASELINE config 4, headline bench.
set -o pipefail
O=gpurun_out/${1:-r4s2}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gemm3_gpu.py tests/test_module_gpu.py tests/test_graphs_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest_sel.log 2>&1 || exit $?
for i in 1 2 3; do
  timeout -k 10 120 python benchmarks/bench_flash.py --only fwd --iters 20 >> $O/fwd_tree.log 2>&1 || exit $?
  XDOT_EXT_PATH=xdot/_C_chainmax.so timeout -k 10 120 python benchmarks/bench_flash.py --only fwd --iters 20 >> $O/fwd_chain.log 2>&1 || exit $?
  timeout -k 10 120 python benchmarks/bench_flash.py --only fwd --iters 20 --R 3125 >> $O/fwd_tree8.log 2>&1 || exit $?
  XDOT_EXT_PATH=xdot/_C_chainmax.so timeout -k 10 120 python benchmarks/bench_flash.py --only fwd --iters 20 --R 3125 >> $O/fwd_chain8.log 2>&1 || exit $?
done
bash scripts/pmc_head.sh ${1:-r4s2}/pmc || exit $?
timeout -k 10 300 python benchmarks/host_step_profile.py --world 8 --steps 40 --inline-backward > $O/host8_inline.log 2>&1 || exit $?
XDOT_FUSED_MODULE=0 timeout -k 10 300 python benchmarks/host_step_profile.py --world 8 --steps 40 --inline-backward > $O/host8_inline_nofuse.log 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 300 python benchmarks/bench_rank.py --world 8 --steps 30 --warmup 5 --fp32-steps 0 >> $O/rank8_fused.log 2>&1 || exit $?
  XDOT_FUSED_MODULE=0 timeout -k 10 300 python benchmarks/bench_rank.py --world 8 --steps 30 --warmup 5 --fp32-steps 0 >> $O/rank8_nofuse.log 2>&1 || exit $?
done
for i in 1 2; do
  timeout -k 10 300 python benchmarks/bench_rank.py --world 8 --rank 3 --steps 30 --warmup 5 --fp32-steps 0 >> $O/rank8_r3.log 2>&1 || exit $?
  timeout -k 10 300 python benchmarks/bench_rank.py --world 8 --rank 3 --no-seg-merge --steps 30 --warmup 5 --fp32-steps 0 >> $O/rank8_r3_nomerge.log 2>&1 || exit $?
done
timeout -k 10 300 python bench.py --seq-len 5000 --steps 50 --warmup 10 --fp32-steps 0 > $O/c2_T5000.log 2>&1 || exit $?
XDOT_FUSED_MODULE=0 timeout -k 10 300 python bench.py --seq-len 5000 --steps 50 --warmup 10 --fp32-steps 0 > $O/c2_T5000_nofuse.log 2>&1 || exit $?
timeout -k 10 200 python benchmarks/bench_ops.py --mode leftT_fb --T 12500 --emulate 8 --dtype fp32 --iters 5 > $O/c4_leftT_fp32.log 2>&1 || exit $?
timeout -k 10 200 python benchmarks/bench_ops.py --mode nt --T 25000 --offset 32 --emulate 8 --dtype fp32 --iters 5 > $O/c3_nt_fp32.log 2>&1 || exit $?
timeout -k 10 200 python benchmarks/bench_ops.py --mode all --T 25000 --offset 32 --emulate 8 --dtype fp32 --iters 5 > $O/c3_all_fp32.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || exit $?
timeout -k 10 300 python benchmarks/bench_rank.py --world 8 --steps 10 --warmup 3 --impl ring --link-gbps 300 --p2p-gbps 64 --fp32-steps 0 > $O/ring8.log 2>&1 || exit $?
XDOT_RING_BIDIR=0 timeout -k 10 300 python benchmarks/bench_rank.py --world 8 --steps 10 --warmup 3 --impl ring --link-gbps 300 --p2p-gbps 64 --fp32-steps 0 > $O/ring8_uni.log 2>&1 || exit $?
bash scripts/gpu_multirank.sh ${1:-r4s2}/mr || exit $?
echo s2-ok
