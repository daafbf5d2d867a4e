#!/bin/bash
# Time split of the default 1M passes (tile-major, pass B 8 rows): loads from one L2-resident
# tile (16), stores dropped (32), both (48). Timing only.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; OUT=$R/gpurun_out; TAG=${1:-c2m2}; mkdir -p $OUT
st() { echo "$1 rc=$2 $(date +%T)" >> $OUT/${TAG}_status.txt; case "$2" in 0) ;; *) exit "$2";; esac; }
echo "start $(date +%T)" > $OUT/${TAG}_status.txt
for v in 0 16 32 48; do
  (cd /tmp && export TMPDIR=/tmp && SDRGPU_TUNING=1 SDRGPU_FFT_1M_VAR=$((128 + v)) SDRGPU_FFT_1M_VARB=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${TAG}_prof_$v -o run -- python3 $R/bench.py --config c2 --no-sub --no-cpu --steps 10 --warmup 2 > $OUT/${TAG}_prof_$v.log 2>&1)
  st prof$v $?
done
echo "all done $(date +%T)" >> $OUT/${TAG}_status.txt
