#!/bin/bash
# per-call kernel traces with the stage-1 rows kernel's history workgroup and/or NCO removed
# (timing probes, wrong results by design)
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; TAG=${1:-rp}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for p in 0 1 2 3; do
  SDRGPU_TUNING=1 SDRGPU_ROWS_PROBE=$p timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${TAG}_$p -o run -- python3 $R/tools/per_call.py 100 single > $OUT/${TAG}_$p.log 2>&1 || exit $?
done
