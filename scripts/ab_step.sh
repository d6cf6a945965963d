#!/bin/bash
# Interleaved step A/B of extension builds / env settings: ab_step.sh OUT REPS "ARGS" spec1 spec2 ...
# spec = path/to/_C_x.so[:VAR=VAL[,VAR2=VAL2]] (loaded through XDOT_EXT_PATH with those env vars);
# bench.py ARGS, e.g. "--dtype fp32 --steps 10 --warmup 3"
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/$1; REPS=$2; ARGS=$3; shift 3
mkdir -p $OUT
for rep in $(seq 1 $REPS); do
  for spec in "$@"; do
    so=${spec%%:*}; envs=""; [[ "$spec" == *:* ]] && envs=${spec#*:}
    n=$(basename $so .so)${envs:+_$(echo $envs | tr ',=' '_-')}
    env ${envs//,/ } XDOT_EXT_PATH=$GRAFT_REPO_ROOT/$so timeout -k 10 300 python bench.py $ARGS --no-check --fp32-steps 0 > $OUT/$n.$rep.log 2>&1 || exit $?
    echo "$n rep $rep: $(grep -o '"ms_per_step": [0-9.]*' $OUT/$n.$rep.log)"
  done
done
