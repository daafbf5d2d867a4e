#!/bin/bash
# Split-frame front end (no stitch copy launch): full -m gpu suite, then per-call A/B against the
# stitching path (SDRGPU_FE_SPLIT=0), then a kernel trace.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; OUT=$R/gpurun_out; TAG=${1:-split}; mkdir -p $OUT
st() { echo "$1 rc=$2 $(date +%T)" >> $OUT/${TAG}_status.txt; case "$2" in 0) ;; *) exit "$2";; esac; }
echo "start $(date +%T)" > $OUT/${TAG}_status.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/${TAG}_tests.log 2>&1
st tests $?
for k in 1 2 3; do
  timeout -k 10 300 python tools/per_call.py 300 single >> $OUT/${TAG}_pc_on.jsonl 2>>$OUT/${TAG}_err.log; st on$k $?
  SDRGPU_TUNING=1 SDRGPU_FE_SPLIT=0 timeout -k 10 300 python tools/per_call.py 300 single >> $OUT/${TAG}_pc_off.jsonl 2>>$OUT/${TAG}_err.log; st off$k $?
done
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${TAG}_trace -o run -- python3 $R/tools/per_call.py 100 single > $OUT/${TAG}_trace.log 2>&1)
st trace $?
echo "all done $(date +%T)" >> $OUT/${TAG}_status.txt
