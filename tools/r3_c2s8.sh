#!/bin/bash
# 1M passes at 8 columns / rows per workgroup (2 workgroups per CU) and XCD-grouped tiles:
# parity tests per configuration, then interleaved C2 benches.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; OUT=$R/gpurun_out; TAG=${1:-c2s}; mkdir -p $OUT
st() { echo "$1 rc=$2 $(date +%T)" >> $OUT/${TAG}_status.txt; case "$2" in 0) ;; *) exit "$2";; esac; }
echo "start $(date +%T)" > $OUT/${TAG}_status.txt
CFGS="${CFGS:-base:16:128:8:64 b16:16:128:16:0 a137:16:137:8:64 rowmaj:16:0:8:64}"
for c in $CFGS; do IFS=: read n sa va sb vb <<< "$c"
  SDRGPU_TUNING=1 SDRGPU_FFT_1M_SA=$sa SDRGPU_FFT_1M_VAR=$va SDRGPU_FFT_1M_SB=$sb SDRGPU_FFT_1M_VARB=$vb timeout -k 10 300 \
    python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "1m or c2 or multi_chunk" > $OUT/${TAG}_tests_$n.log 2>&1
  st tests_$n $?
done
for rep in 1 2 3; do for c in $CFGS; do IFS=: read n sa va sb vb <<< "$c"
  SDRGPU_TUNING=1 SDRGPU_FFT_1M_SA=$sa SDRGPU_FFT_1M_VAR=$va SDRGPU_FFT_1M_SB=$sb SDRGPU_FFT_1M_VARB=$vb timeout -k 10 300 \
    python bench.py --config c2 --steps 20 --no-cpu --no-sub >> $OUT/${TAG}_c2_$n.jsonl 2>>$OUT/${TAG}_err.log; st c2_${n}_$rep $?
done; done
echo "all done $(date +%T)" >> $OUT/${TAG}_status.txt
