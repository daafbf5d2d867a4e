#!/bin/bash
# SQ counters per dispatch of the per-call (307,200-sample block) launch sequence
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; TAG=${1:-pcp}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_WAIT_ANY SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $OUT/${TAG}_$i -o run -- python3 $R/tools/per_call.py 30 single > $OUT/${TAG}_$i.log 2>&1
  rc=$?; echo "set $i rc=$rc" >> $OUT/${TAG}_status.txt
  [ $rc -ne 0 ] && exit $rc
done
echo done >> $OUT/${TAG}_status.txt
