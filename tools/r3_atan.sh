#!/bin/bash
# polynomial quadrature atan2: every -m gpu test, then C3 / C5 bench A/B against the OCML build (lib_old)
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; OUT=$R/gpurun_out; TAG=${1:-at}; mkdir -p $OUT
st() { echo "$1 rc=$2 $(date +%T)" >> $OUT/${TAG}_status.txt; case "$2" in 0) ;; *) exit "$2";; esac; }
echo "start $(date +%T)" > $OUT/${TAG}_status.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/${TAG}_tests.log 2>&1
st tests $?
timeout -k 10 400 bash tools/ab_lib.sh ${TAG}_c3 c3; st ab_c3 $?
timeout -k 10 400 bash tools/ab_lib.sh ${TAG}_c5 c5; st ab_c5 $?
echo "all done $(date +%T)" >> $OUT/${TAG}_status.txt
