#!/bin/bash
# C2: non-temporal dB row stores in pass B (SDRGPU_FFT_1M = 5) vs the default: the 1M parity tests in
# that mode, then 3 interleaved bench runs each
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; OUT=$R/gpurun_out; TAG=${1:-nts}; mkdir -p $OUT
st() { echo "$1 rc=$2 $(date +%T)" >> $OUT/${TAG}_status.txt; case "$2" in 0) ;; *) exit "$2";; esac; }
echo "start $(date +%T)" > $OUT/${TAG}_status.txt
SDRGPU_TUNING=1 SDRGPU_FFT_1M=5 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider -k "1M or c2 or 1m or ulp" --timeout 120 --timeout-method thread > $OUT/${TAG}_tests_5.log 2>&1
st tests_5 $?
for k in 1 2 3; do for m in 1 5; do
  SDRGPU_TUNING=1 SDRGPU_FFT_1M=$m timeout -k 10 200 python bench.py --config c2 --no-sub --no-cpu --steps 20 --warmup 3 >> $OUT/${TAG}_c2_$m.jsonl 2>>$OUT/${TAG}_err.log
  st b_${m}_$k $?
done; done
echo "all done $(date +%T)" >> $OUT/${TAG}_status.txt
