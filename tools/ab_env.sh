#!/bin/bash
# A/B of one tuning setting on one box, interleaved: the default build vs the same build with
# SDRGPU_TUNING=1 and the given variable set.  usage: TAG=x CFGS="c3" REPS=3 bash tools/ab_env.sh VAR=value
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; OUT=$R/gpurun_out; mkdir -p $OUT
SET=$1; TAG=${TAG:-abenv}
for rep in $(seq 1 ${REPS:-3}); do
  for cfg in ${CFGS:-c3}; do
    timeout -k 10 300 python bench.py --config $cfg --steps ${STEPS:-20} --no-cpu --no-sub > $OUT/${TAG}_${cfg}_dflt_$rep.json 2>&1 || exit $?
    env SDRGPU_TUNING=1 $SET timeout -k 10 300 python bench.py --config $cfg --steps ${STEPS:-20} --no-cpu --no-sub > $OUT/${TAG}_${cfg}_env_$rep.json 2>&1 || exit $?
  done
done
