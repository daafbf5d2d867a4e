#!/bin/bash
# C2 tile-major passes with non-temporal input loads (SDRGPU_FFT_1M = 3) and + pass B (= 4) vs the default:
# the parity tests of the 1M path under each mode, then 3 interleaved bench runs each, and PMC FETCH per mode
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; OUT=$R/gpurun_out; TAG=${1:-nt}; mkdir -p $OUT
st() { echo "$1 rc=$2 $(date +%T)" >> $OUT/${TAG}_status.txt; case "$2" in 0) ;; *) exit "$2";; esac; }
echo "start $(date +%T)" > $OUT/${TAG}_status.txt
for m in 3 4; do
  SDRGPU_TUNING=1 SDRGPU_FFT_1M=$m timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider -k "1M or c2 or 1m or ulp" --timeout 120 --timeout-method thread > $OUT/${TAG}_tests_$m.log 2>&1
  st tests_$m $?
done
for k in 1 2 3; do for m in 1 3 4; do
  SDRGPU_TUNING=1 SDRGPU_FFT_1M=$m timeout -k 10 200 python bench.py --config c2 --no-sub --no-cpu --steps 20 --warmup 3 >> $OUT/${TAG}_c2_$m.jsonl 2>>$OUT/${TAG}_err.log
  st b_${m}_$k $?
done; done
for m in 1 3; do
  (cd /tmp && export TMPDIR=/tmp && SDRGPU_TUNING=1 SDRGPU_FFT_1M=$m timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/${TAG}_pmc_$m -o run -- python3 $R/bench.py --config c2 --no-sub --no-cpu --steps 3 --warmup 1 > $OUT/${TAG}_pmc_$m.log 2>&1)
  st pmc_$m $?
done
echo "all done $(date +%T)" >> $OUT/${TAG}_status.txt
