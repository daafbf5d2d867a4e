#!/bin/bash
# packed-asm cmul A/B: C2 / C5 / C4 bench against the previous build (lib_old), interleaved
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; OUT=$R/gpurun_out; TAG=${1:-cm}; mkdir -p $OUT
st() { echo "$1 rc=$2 $(date +%T)" >> $OUT/${TAG}_status.txt; case "$2" in 0) ;; *) exit "$2";; esac; }
echo "start $(date +%T)" > $OUT/${TAG}_status.txt
for c in c2 c5 c4; do timeout -k 10 400 bash tools/ab_lib.sh ${TAG}_$c $c; st ab_$c $?; done
echo "all done $(date +%T)" >> $OUT/${TAG}_status.txt
