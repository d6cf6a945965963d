#!/bin/bash
# Round-4 session 2b: bench.py with stage tracing (and a faulthandler traceback dump of every
# thread if it stalls), then the rest of session 2 when it completes.
set -o pipefail
T=${1:-r4s2b}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 170 python -X faulthandler -c "import faulthandler, sys; f = open('$O/tb.txt', 'w'); faulthandler.dump_traceback_later(140, exit=True, file=f); sys.argv = ['bench.py', '--steps', '20', '--warmup', '5', '--trace']; import runpy; runpy.run_path('bench.py', run_name='__main__')" > $O/bench_trace.log 2>&1 || exit $?
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
bash scripts/gpu_multirank.sh $T/mr || exit $?
echo s2b-ok
