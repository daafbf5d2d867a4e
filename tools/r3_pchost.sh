#!/bin/bash
# Per-call host issue time vs device time: Python (per_call.py) and native C++ (tools/bin/per_call_cpp),
# plus a kernel trace of the native run.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; OUT=$R/gpurun_out; TAG=${1:-pch}; mkdir -p $OUT
st() { echo "$1 rc=$2 $(date +%T)" >> $OUT/${TAG}_status.txt; case "$2" in 0) ;; *) exit "$2";; esac; }
echo "start $(date +%T)" > $OUT/${TAG}_status.txt
for k in 1 2; do
  timeout -k 10 300 python tools/per_call.py 300 single >> $OUT/${TAG}_py.jsonl 2>>$OUT/${TAG}_err.log; st py$k $?
  timeout -k 10 120 tools/bin/per_call_cpp 2000 >> $OUT/${TAG}_cpp.jsonl 2>>$OUT/${TAG}_err.log; st cpp$k $?
done
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/${TAG}_trace -o run -- $R/tools/bin/per_call_cpp 300 > $OUT/${TAG}_trace.log 2>&1)
st trace $?
echo "all done $(date +%T)" >> $OUT/${TAG}_status.txt
