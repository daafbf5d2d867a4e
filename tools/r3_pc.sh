#!/bin/bash
# per-call check: every -m gpu test, then per_call (single stream) with the FIR tail on / off, and a
# kernel trace of the per-call launch sequence
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; OUT=$R/gpurun_out; TAG=${1:-pc}; mkdir -p $OUT
st() { echo "$1 rc=$2 $(date +%T)" >> $OUT/${TAG}_status.txt; case "$2" in 0) ;; *) exit "$2";; esac; }
echo "start $(date +%T)" > $OUT/${TAG}_status.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/${TAG}_tests.log 2>&1
st tests $?
for k in 1 2; do
  timeout -k 10 120 python tools/per_call.py 300 single >> $OUT/${TAG}_pc.jsonl 2>> $OUT/${TAG}_pc.err; st pc_on_$k $?
  SDRGPU_TUNING=1 SDRGPU_VFO_TAIL=0 timeout -k 10 120 python tools/per_call.py 300 single >> $OUT/${TAG}_pc_off.jsonl 2>> $OUT/${TAG}_pc.err; st pc_off_$k $?
done
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/${TAG}_pct -o run -- python3 $R/tools/per_call.py 60 single > $OUT/${TAG}_pct.log 2>&1)
st pct $?
echo "all done $(date +%T)" >> $OUT/${TAG}_status.txt
