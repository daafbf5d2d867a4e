#!/bin/bash
# Env-variant sweep of bench.py on one box: TAG=x CFG=c3 bash tools/sweep.sh 'ENV1=a ENV2=b' 'ENV3=c' ...
# (an empty string = defaults). Stops at the first failure.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; OUT=$R/gpurun_out; mkdir -p $OUT
i=0
for v in "$@"; do
  i=$((i+1))
  env $v timeout -k 10 300 python bench.py --config ${CFG:-c3} --steps ${STEPS:-20} --no-cpu > $OUT/${TAG}_${CFG}_$i.json 2>&1 || exit $?
  echo "$i $v" >> $OUT/${TAG}_${CFG}_legend.txt
done
