#!/bin/bash
# packed-asm cmul: every -m gpu test, then C2 / C5 / C4 bench A/B against the previous build (lib_old)
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; OUT=$R/gpurun_out; TAG=${1:-cm}; mkdir -p $OUT
st() { echo "$1 rc=$2 $(date +%T)" >> $OUT/${TAG}_status.txt; case "$2" in 0) ;; *) exit "$2";; esac; }
echo "start $(date +%T)" > $OUT/${TAG}_status.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/${TAG}_tests.log 2>&1
st tests $?
for c in c2 c5 c4; do timeout -k 10 400 bash tools/ab_lib.sh ${TAG}_$c $c; st ab_$c $?; done
echo "all done $(date +%T)" >> $OUT/${TAG}_status.txt
