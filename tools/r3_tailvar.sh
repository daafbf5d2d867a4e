#!/bin/bash
# fir_tail_kernel time split: kernel trace of per_call with SDRGPU_TAIL_VAR = 0 (full), 1 (no stage
# loops), 2 (no image loads) -- timing only, variants 1 and 2 give wrong results
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; OUT=$R/gpurun_out; TAG=${1:-tv}; mkdir -p $OUT
st() { echo "$1 rc=$2 $(date +%T)" >> $OUT/${TAG}_status.txt; case "$2" in 0) ;; *) exit "$2";; esac; }
echo "start $(date +%T)" > $OUT/${TAG}_status.txt
for v in 0 1 2; do
(cd /tmp && export TMPDIR=/tmp && SDRGPU_TUNING=1 SDRGPU_TAIL_VAR=$v timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/${TAG}_v$v -o run -- python3 $R/tools/per_call.py 60 single > $OUT/${TAG}_v$v.log 2>&1)
st v$v $?
done
echo "all done $(date +%T)" >> $OUT/${TAG}_status.txt
