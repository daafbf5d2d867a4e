#!/bin/bash
# Round-3 C3 iteration: DDC tests (fast-convolution default) then interleaved A/B of the fast
# convolution against the matrix-core FIR (SDRGPU_FIR_FFTCONV=0), and a kernel-stats profile.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; OUT=$R/gpurun_out; TAG=${1:-c3}; mkdir -p $OUT
st() { echo "$1 rc=$2 $(date +%T)" >> $OUT/${TAG}_status.txt; case "$2" in 0) ;; *) exit "$2";; esac; }
echo "start $(date +%T)" > $OUT/${TAG}_status.txt
SDRGPU_REPORT_DIR=$OUT/${TAG}_rep timeout -k 10 300 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  -k "ddc or c3" > $OUT/${TAG}_tests.log 2>&1
echo "tests rc=$? $(date +%T)" >> $OUT/${TAG}_status.txt
for rep in 1 2; do
  timeout -k 10 300 python bench.py --config c3 --steps 20 --no-cpu --no-sub > $OUT/${TAG}_new_$rep.json 2>&1; st new$rep $?
  SDRGPU_TUNING=1 SDRGPU_FIR_FFTCONV=0 timeout -k 10 300 python bench.py --config c3 --steps 20 --no-cpu --no-sub > $OUT/${TAG}_old_$rep.json 2>&1; st old$rep $?
done
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${TAG}_prof -o run -- python3 $R/bench.py --config c3 --no-sub --no-cpu --steps 10 --warmup 2 > $OUT/${TAG}_prof.log 2>&1)
st prof $?
echo "all done $(date +%T)" >> $OUT/${TAG}_status.txt
