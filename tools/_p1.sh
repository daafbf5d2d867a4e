#!/bin/bash
# pass-A timing ablations (64k): rocprofv3 kernel stats per SDRGPU_FFT_DEBUG value
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for d in ${DBGS:-0 1 2 3 16 17 19 0}; do
  SDRGPU_FFT_DEBUG=$d timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/p1_$d -o run -- python3 $R/tools/fft_one.py ${N:-65536} ${NZ:-65536} ${FR:-4096} 6 > $OUT/p1_$d.log 2>&1 || exit $?
  grep -h "fft_pass" $OUT/p1_$d/run_kernel_stats.csv | awk -F'",' -v d=$d '{print d, substr($1,1,40), $0}' | awk -F, '{print $1, $(NF-4)}' >> $OUT/p1_summary.txt
done
