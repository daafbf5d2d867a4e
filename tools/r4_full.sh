#!/bin/bash
# Full GPU session: every -m gpu test, smoke, the default bench (CPU legs included), per-call trace,
# rocprofv3 kernel stats per config and FETCH/WRITE PMC passes for C2 and C5.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; OUT=$R/gpurun_out; TAG=${1:-full}; mkdir -p $OUT
st() { echo "$1 rc=$2 $(date +%T)" >> $OUT/${TAG}_status.txt; case "$2" in 0) ;; *) exit "$2";; esac; }
echo "start $(date +%T)" > $OUT/${TAG}_status.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/${TAG}_tests.log 2>&1
st tests $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/${TAG}_smoke.log 2>&1
st smoke $?
timeout -k 10 600 python bench.py > $OUT/${TAG}_bench.json 2> $OUT/${TAG}_bench.err
st bench $?
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/${TAG}_pct -o run -- python3 $R/tools/per_call.py 60 single > $OUT/${TAG}_pct.log 2>&1)
st pct $?
for c in c5 c2 c3 c4 c4g; do
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${TAG}_prof_$c -o run -- python3 $R/bench.py --config $c --no-sub --no-cpu --steps 10 --warmup 2 > $OUT/${TAG}_prof_$c.log 2>&1)
  st prof_$c $?
done
for c in c2 c5 c3; do for ctr in FETCH_SIZE WRITE_SIZE; do
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $OUT/${TAG}_pmc_${c}_$ctr -o run -- python3 $R/bench.py --config $c --no-sub --no-cpu --steps 3 --warmup 1 > $OUT/${TAG}_pmc_${c}_$ctr.log 2>&1)
  st pmc_${c}_$ctr $?
done; done
echo "all done $(date +%T)" >> $OUT/${TAG}_status.txt
