#!/bin/bash
# 64k pass A streaming input loads (SDRGPU_PA_CP = 2, this build) vs cached (lib_old): every -m gpu test,
# then the C5 bench A/B, 3 interleaved runs
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; OUT=$R/gpurun_out; TAG=${1:-pa}; mkdir -p $OUT
st() { echo "$1 rc=$2 $(date +%T)" >> $OUT/${TAG}_status.txt; case "$2" in 0) ;; *) exit "$2";; esac; }
echo "start $(date +%T)" > $OUT/${TAG}_status.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/${TAG}_tests.log 2>&1
st tests $?
timeout -k 10 400 bash tools/ab_lib.sh ${TAG}_${CFG:-c5} ${CFG:-c5}; st ab $?
echo "all done $(date +%T)" >> $OUT/${TAG}_status.txt
