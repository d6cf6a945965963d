#!/bin/bash
# Round-4 session 2 (one call, most important first): full GPU suite + smoke, forward row-max A/B
# (tree vs chain), HEAD PMC table of the flash kernels, host profiles (fused module node vs per-op
# graph), emulated N=8 rank steps (rank 0 / middle rank 3 with and without the merged segments),
# BASELINE config 2 (T=5000), ring N=8 (bidirectional vs one-way), headline bench, exact-fp32
# configs, multi-rank gloo rehearsals.  Every GPU step has its own time limit.
set -o pipefail
O=gpurun_out/${1:-r4s2}
mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke-ok')" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -rf > $O/pytest.log 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 120 python benchmarks/bench_flash.py --only fwd --iters 20 >> $O/fwd_tree.log 2>&1 || exit $?
  XDOT_EXT_PATH=xdot/_C_chainmax.so timeout -k 10 120 python benchmarks/bench_flash.py --only fwd --iters 20 >> $O/fwd_chain.log 2>&1 || exit $?
  timeout -k 10 120 python benchmarks/bench_flash.py --only fwd --iters 20 --R 3125 >> $O/fwd_tree8.log 2>&1 || exit $?
  XDOT_EXT_PATH=xdot/_C_chainmax.so timeout -k 10 120 python benchmarks/bench_flash.py --only fwd --iters 20 --R 3125 >> $O/fwd_chain8.log 2>&1 || exit $?
done
bash scripts/pmc_head.sh ${1:-r4s2}/pmc || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || exit $?
timeout -k 10 300 python benchmarks/host_step_profile.py --world 8 --steps 40 --inline-backward > $O/host8_inline.log 2>&1 || exit $?
XDOT_FUSED_MODULE=0 timeout -k 10 300 python benchmarks/host_step_profile.py --world 8 --steps 40 > $O/host8_nofuse.log 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 300 python benchmarks/bench_rank.py --world 8 --steps 30 --warmup 5 --fp32-steps 0 >> $O/rank8_fused.log 2>&1 || exit $?
  XDOT_FUSED_MODULE=0 timeout -k 10 300 python benchmarks/bench_rank.py --world 8 --steps 30 --warmup 5 --fp32-steps 0 >> $O/rank8_nofuse.log 2>&1 || exit $?
  timeout -k 10 300 python benchmarks/bench_rank.py --world 8 --rank 3 --steps 30 --warmup 5 --fp32-steps 0 >> $O/rank8_r3.log 2>&1 || exit $?
  timeout -k 10 300 python benchmarks/bench_rank.py --world 8 --rank 3 --no-seg-merge --steps 30 --warmup 5 --fp32-steps 0 >> $O/rank8_r3_nomerge.log 2>&1 || exit $?
done
timeout -k 10 300 python bench.py --seq-len 5000 --steps 50 --warmup 10 --fp32-steps 0 > $O/c2_T5000.log 2>&1 || exit $?
XDOT_FUSED_MODULE=0 timeout -k 10 300 python bench.py --seq-len 5000 --steps 50 --warmup 10 --fp32-steps 0 > $O/c2_T5000_nofuse.log 2>&1 || exit $?
timeout -k 10 300 python benchmarks/bench_rank.py --world 8 --steps 10 --warmup 3 --impl ring --link-gbps 300 --p2p-gbps 64 --fp32-steps 0 > $O/ring8.log 2>&1 || exit $?
XDOT_RING_BIDIR=0 timeout -k 10 300 python benchmarks/bench_rank.py --world 8 --steps 10 --warmup 3 --impl ring --link-gbps 300 --p2p-gbps 64 --fp32-steps 0 > $O/ring8_uni.log 2>&1 || exit $?
timeout -k 10 200 python benchmarks/bench_ops.py --mode leftT_fb --T 12500 --emulate 8 --dtype fp32 --iters 5 > $O/c4_leftT_fp32.log 2>&1 || exit $?
timeout -k 10 200 python benchmarks/bench_ops.py --mode nt --T 25000 --offset 32 --emulate 8 --dtype fp32 --iters 5 > $O/c3_nt_fp32.log 2>&1 || exit $?
timeout -k 10 200 python benchmarks/bench_ops.py --mode all --T 25000 --offset 32 --emulate 8 --dtype fp32 --iters 5 > $O/c3_all_fp32.log 2>&1 || exit $?
bash scripts/gpu_multirank.sh ${1:-r4s2}/mr || exit $?
echo s2-ok
