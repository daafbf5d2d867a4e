#!/bin/bash
# A/B timing of the in-tree build against abtest/libsdrgpu_<B>.so on one box, interleaved.
# usage: TAG=x CFGS="c3 c5" REPS=2 bash tools/ab.sh B
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; OUT=$R/gpurun_out; mkdir -p $OUT
B=${1:-r0}; TAG=${TAG:-ab}
for rep in $(seq 1 ${REPS:-2}); do
  for cfg in ${CFGS:-c3 c5}; do
    timeout -k 10 300 python bench.py --config $cfg --steps ${STEPS:-20} --no-cpu > $OUT/${TAG}_${cfg}_new_$rep.json 2>&1 || exit $?
    SDRGPU_LIB_PATH=$R/abtest/libsdrgpu_$B.so timeout -k 10 300 python bench.py --config $cfg --steps ${STEPS:-20} --no-cpu > $OUT/${TAG}_${cfg}_${B}_$rep.json 2>&1 || exit $?
  done
done
