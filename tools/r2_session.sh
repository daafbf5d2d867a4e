#!/bin/bash
# Round-2 GPU session: GPU tests (reports to gpurun_out/<tag>_rep) -> default bench line ->
# rocprofv3 kernel stats per config -> PMC FETCH/WRITE passes per config. Stops at the first
# crash / timeout (rc 124/134/137/139); a failing test run stops the session too.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; OUT=$R/gpurun_out; TAG=${1:-r2}; mkdir -p $OUT
st() { echo "$1 rc=$2 $(date +%T)" >> $OUT/${TAG}_status.txt; case "$2" in 0) ;; *) exit "$2";; esac; }
echo "start $(date +%T)" > $OUT/${TAG}_status.txt
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  SDRGPU_REPORT_DIR=$OUT/${TAG}_rep timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/${TAG}_tests.log 2>&1
  st tests $?
fi
if [ "${SKIP_BENCH:-0}" != "1" ]; then
  timeout -k 10 600 python bench.py > $OUT/${TAG}_bench.json 2> $OUT/${TAG}_bench.err
  st bench $?
fi
for cfg in ${PROF_CFGS:-c5 c2 c3 c4}; do
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${TAG}_prof_$cfg -o run -- python3 $R/bench.py --config $cfg --no-sub --no-cpu --steps 10 --warmup 2 > $OUT/${TAG}_prof_$cfg.log 2>&1)
  st prof_$cfg $?
done
for cfg in ${PMC_CFGS:-c5 c2}; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $OUT/${TAG}_pmc_${cfg}_$ctr -o run -- python3 $R/bench.py --config $cfg --no-sub --no-cpu --steps 3 --warmup 1 > $OUT/${TAG}_pmc_${cfg}_$ctr.log 2>&1)
    st pmc_${cfg}_$ctr $?
  done
done
echo "all done $(date +%T)" >> $OUT/${TAG}_status.txt
