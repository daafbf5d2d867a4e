#!/bin/bash
# kernel trace of the per-call (307,200-sample block) launch sequence, tail chain on / off
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; TAG=${1:-pct}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/${TAG}_on -o run -- python3 $R/tools/per_call.py 60 single > $OUT/${TAG}_on.log 2>&1 || exit 1
SDRGPU_TUNING=1 SDRGPU_VFO_TAIL=0 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/${TAG}_off -o run -- python3 $R/tools/per_call.py 60 single > $OUT/${TAG}_off.log 2>&1
