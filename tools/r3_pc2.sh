#!/bin/bash
# per-call launch interleaving: every -m gpu test (default mode), then per_call (single stream) with
# SDRGPU_FE_INTERLEAVE = 0 / 1 / 2 interleaved twice, and a kernel trace of modes 1 and 2
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; OUT=$R/gpurun_out; TAG=${1:-pc2}; mkdir -p $OUT
st() { echo "$1 rc=$2 $(date +%T)" >> $OUT/${TAG}_status.txt; case "$2" in 0) ;; *) exit "$2";; esac; }
echo "start $(date +%T)" > $OUT/${TAG}_status.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/${TAG}_tests.log 2>&1
st tests $?
for k in 1 2; do for m in 0 1 2; do
  SDRGPU_TUNING=1 SDRGPU_FE_INTERLEAVE=$m timeout -k 10 120 python tools/per_call.py 300 single | sed "s/^/{\"mode\": $m, \"r\": /; s/$/}/" >> $OUT/${TAG}_pc.jsonl 2>> $OUT/${TAG}_pc.err; st pc_${m}_$k $?
done; done
for m in 1 2; do
(cd /tmp && export TMPDIR=/tmp && SDRGPU_TUNING=1 SDRGPU_FE_INTERLEAVE=$m timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/${TAG}_pct$m -o run -- python3 $R/tools/per_call.py 60 single > $OUT/${TAG}_pct$m.log 2>&1)
st pct$m $?
done
echo "all done $(date +%T)" >> $OUT/${TAG}_status.txt
