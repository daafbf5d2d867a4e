#!/bin/bash
# Round-3 C2 iteration 2: 1M spectrum tests, the C2 bench twice, a kernel-stats profile.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; OUT=$R/gpurun_out; TAG=${1:-c2b}; mkdir -p $OUT
st() { echo "$1 rc=$2 $(date +%T)" >> $OUT/${TAG}_status.txt; case "$2" in 0) ;; *) exit "$2";; esac; }
echo "start $(date +%T)" > $OUT/${TAG}_status.txt
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  -k "fft or spectrum or c2 or 1m or 1M" > $OUT/${TAG}_tests.log 2>&1
st tests $?
for rep in 1 2; do
  timeout -k 10 300 python bench.py --config c2 --steps 20 --no-cpu --no-sub > $OUT/${TAG}_c2_$rep.json 2>&1; st c2_$rep $?
done
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${TAG}_prof -o run -- python3 $R/bench.py --config c2 --no-sub --no-cpu --steps 10 --warmup 2 > $OUT/${TAG}_prof.log 2>&1)
st prof $?
echo "all done $(date +%T)" >> $OUT/${TAG}_status.txt
