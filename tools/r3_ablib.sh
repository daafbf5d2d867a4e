#!/bin/bash
# A/B of two builds of libsdrgpu on one box: abtmp/libsdrgpu_base.so vs sdrpp_amd/lib/libsdrgpu.so.
# The new build's full -m gpu suite first, then interleaved benches of the configs given ($2..).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; OUT=$R/gpurun_out; TAG=${1:-ab}; shift; CFGS=${@:-c5 c2}; mkdir -p $OUT
st() { echo "$1 rc=$2 $(date +%T)" >> $OUT/${TAG}_status.txt; case "$2" in 0) ;; *) exit "$2";; esac; }
echo "start $(date +%T)" > $OUT/${TAG}_status.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/${TAG}_tests.log 2>&1
st tests $?
for k in 1 2 3; do for c in $CFGS; do for v in base new; do
  if [ $v == base ]; then L=$R/abtmp/libsdrgpu_base.so; else L=$R/sdrpp_amd/lib/libsdrgpu.so; fi
  SDRGPU_LIB_PATH=$L timeout -k 10 200 python bench.py --config $c --no-sub --no-cpu --steps 20 --warmup 3 >> $OUT/${TAG}_${c}_$v.jsonl 2>>$OUT/${TAG}_err.log
  st ${c}_${v}_$k $?
done; done; done
echo "all done $(date +%T)" >> $OUT/${TAG}_status.txt
