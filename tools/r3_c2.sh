#!/bin/bash
# Round-3 C2 iteration: 1M spectrum tests on the default build, then interleaved A/B of the
# persistent pipelined 1M passes (default) against the one-shot passes (SDRGPU_FFT_1M=0), and of
# the per-call cost with / without the StreamOrder end-of-call event (SDRGPU_ORDER_DONE=0).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; OUT=$R/gpurun_out; TAG=${1:-c2}; mkdir -p $OUT
st() { echo "$1 rc=$2 $(date +%T)" >> $OUT/${TAG}_status.txt; case "$2" in 0) ;; *) exit "$2";; esac; }
echo "start $(date +%T)" > $OUT/${TAG}_status.txt
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  -k "fft or spectrum or c2 or 1m or 1M" > $OUT/${TAG}_tests.log 2>&1
st tests $?
for rep in 1 2; do
  timeout -k 10 300 python bench.py --config c2 --steps 20 --no-cpu --no-sub > $OUT/${TAG}_new_$rep.json 2>&1; st new$rep $?
  SDRGPU_TUNING=1 SDRGPU_FFT_1M=0 timeout -k 10 300 python bench.py --config c2 --steps 20 --no-cpu --no-sub > $OUT/${TAG}_old_$rep.json 2>&1; st old$rep $?
done
for rep in 1 2; do
  timeout -k 10 300 python tools/per_call.py 300 single > $OUT/${TAG}_pc_done_$rep.json 2>&1; st pcd$rep $?
  SDRGPU_TUNING=1 SDRGPU_ORDER_DONE=0 timeout -k 10 300 python tools/per_call.py 300 single > $OUT/${TAG}_pc_nodone_$rep.json 2>&1; st pcn$rep $?
done
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${TAG}_prof -o run -- python3 $R/bench.py --config c2 --no-sub --no-cpu --steps 10 --warmup 2 > $OUT/${TAG}_prof.log 2>&1)
st prof $?
echo "all done $(date +%T)" >> $OUT/${TAG}_status.txt
