#!/bin/bash
# Bisect the fp32-exact step stall seen in r4s2 / r4s2b: each variant in its own process under a
# time limit with a faulthandler traceback dump; the first stall ends the script.
set -o pipefail
T=${1:-r4dbg}
O=gpurun_out/$T
mkdir -p $O
run() {  # name, env...
  name=$1; shift
  env "$@" timeout -k 10 130 python -X faulthandler -c "import faulthandler, sys; f = open('$O/tb_$name.txt', 'w'); faulthandler.dump_traceback_later(100, exit=True, file=f); sys.argv = ['bench.py', '--steps', '2', '--warmup', '1', '--fp32-steps', '2', '--fp32-warmup', '1', '--no-check', '--trace']; import runpy; runpy.run_path('bench.py', run_name='__main__')" > $O/$name.log 2>&1
}
run noside XDOT_WGRAD_SIDE=0 || exit $?
run nofuse XDOT_FUSED_MODULE=0 || exit $?
echo dbg-ok
