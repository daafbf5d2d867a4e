#!/bin/bash
# 1M pass-A variants (SDRGPU_FFT_1M_VAR): parity tests per variant, then interleaved C2 benches.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; OUT=$R/gpurun_out; TAG=${1:-c2v}; shift; VARS=${@:-0 8 9 12 13 15}; mkdir -p $OUT
st() { echo "$1 rc=$2 $(date +%T)" >> $OUT/${TAG}_status.txt; case "$2" in 0) ;; *) exit "$2";; esac; }
echo "start $(date +%T)" > $OUT/${TAG}_status.txt
for v in $VARS; do
  SDRGPU_TUNING=1 SDRGPU_FFT_1M_VAR=$v timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
    -k "1m or c2 or multi_chunk" > $OUT/${TAG}_tests_$v.log 2>&1
  st tests$v $?
done
for rep in 1 2 3; do for v in $VARS; do
  SDRGPU_TUNING=1 SDRGPU_FFT_1M_VAR=$v timeout -k 10 300 python bench.py --config c2 --steps 20 --no-cpu --no-sub >> $OUT/${TAG}_c2_$v.jsonl 2>>$OUT/${TAG}_err.log; st c2_${v}_$rep $?
done; done
echo "all done $(date +%T)" >> $OUT/${TAG}_status.txt
