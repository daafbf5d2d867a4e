#!/bin/bash
# packed-asm cmulf (NCO rotation in the FIR kernels): every -m gpu test, then C3 / C5 A/B vs lib_old
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; OUT=$R/gpurun_out; TAG=${1:-cf}; mkdir -p $OUT
st() { echo "$1 rc=$2 $(date +%T)" >> $OUT/${TAG}_status.txt; case "$2" in 0) ;; *) exit "$2";; esac; }
echo "start $(date +%T)" > $OUT/${TAG}_status.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/${TAG}_tests.log 2>&1
st tests $?
for c in c3 c5; do timeout -k 10 400 bash tools/ab_lib.sh ${TAG}_$c $c; st ab_$c $?; done
for k in 1 2; do
  SDRGPU_LIB_PATH=$R/sdrpp_amd/lib_old/libsdrgpu.so timeout -k 10 120 python tools/per_call.py 300 single >> $OUT/${TAG}_pc_old.jsonl 2>> $OUT/${TAG}_pc.err; st pc_old_$k $?
  timeout -k 10 120 python tools/per_call.py 300 single >> $OUT/${TAG}_pc_new.jsonl 2>> $OUT/${TAG}_pc.err; st pc_new_$k $?
done
echo "all done $(date +%T)" >> $OUT/${TAG}_status.txt
