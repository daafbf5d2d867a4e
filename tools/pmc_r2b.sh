#!/bin/bash
# Round-2 counter passes beyond FETCH/WRITE: C3's MFMA FIR issue picture (MFMA busy, wait / issue
# stalls, LDS) and, for C5 / C2, how many of the L2's memory-side requests go to DRAM.
# One rocprofv3 --pmc pass per counter set (SQ <= 8, TCC <= 4, GRBM <= 2 per pass).
# usage: bash tools/pmc_r2b.sh TAG   -> gpurun_out/TAG_<name>/ ; summarise with tools/pmc_summary.py
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; TAG=${1:-r2b}; mkdir -p $OUT
echo "start $(date +%T)" > $OUT/${TAG}_status.txt
run() {   # name cfg regex counters...
  local name=$1 cfg=$2 rx=$3; shift 3
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace --kernel-include-regex "$rx" \
     --output-format csv -d $OUT/${TAG}_$name -o run -- python3 $R/bench.py --config $cfg --no-sub --no-cpu --steps 3 --warmup 1 \
     > $OUT/${TAG}_$name.log 2>&1)
  local rc=$?; echo "$name rc=$rc $(date +%T)" >> $OUT/${TAG}_status.txt
  [ $rc -eq 0 ] || exit $rc
}
run c3_mfma c3 fir_mfma SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE
run c3_issue c3 fir_mfma SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_MFMA SQ_WAVES SQ_VALU_MFMA_COEXEC_CYCLES GRBM_GUI_ACTIVE
run c5_rd c5 . TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum GRBM_GUI_ACTIVE
run c5_wr c5 . TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_DRAM_sum GRBM_GUI_ACTIVE
run c2_rd c2 . TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum GRBM_GUI_ACTIVE
echo "all done $(date +%T)" >> $OUT/${TAG}_status.txt
