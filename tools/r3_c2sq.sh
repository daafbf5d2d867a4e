#!/bin/bash
# SQ counters for the 1M passes (C2 bench, 3 steps): issue / wait breakdown of pass A and pass B.
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; TAG=${1:-c2sq}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" "SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $OUT/${TAG}_$i -o run -- python3 $R/bench.py --config c2 --no-sub --no-cpu --steps 3 --warmup 1 > $OUT/${TAG}_$i.log 2>&1
  rc=$?; echo "set $i rc=$rc" >> $OUT/${TAG}_status.txt
  [ $rc -ne 0 ] && exit $rc
done
echo done >> $OUT/${TAG}_status.txt
