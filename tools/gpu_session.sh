#!/bin/bash
# One GPU-box session: parity tests -> bench lines -> rocprofv3 kernel trace.
# Stops at the first crash/timeout (rc 124/134/137/139): nothing else runs on the GPU after that.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=$R/gpurun_out
TAG=${1:-s}
mkdir -p "$OUT"
fatal() { case "$1" in 124|134|137|139) echo "FATAL rc=$1 at $2" >> "$OUT/${TAG}_status.txt"; exit "$1";; esac; }
echo "start $(date)" > "$OUT/${TAG}_status.txt"
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -q --timeout 300 -p no:cacheprovider > "$OUT/${TAG}_gpu_tests.log" 2>&1
  rc=$?; echo "tests rc=$rc" >> "$OUT/${TAG}_status.txt"; fatal $rc tests
fi
for cfg in ${BENCH_CFGS:-c5 c3 c2}; do
  timeout -k 10 400 python bench.py --config $cfg --no-sub --steps ${STEPS:-20} --warmup 3 --cpu-seconds ${CPUSEC:-6} > "$OUT/${TAG}_bench_$cfg.json" 2> "$OUT/${TAG}_bench_$cfg.err"
  rc=$?; echo "bench $cfg rc=$rc" >> "$OUT/${TAG}_status.txt"; fatal $rc bench_$cfg
done
if [ "${PROFILE:-1}" == "1" ]; then
  for cfg in ${PROF_CFGS:-c5}; do
    (cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${TAG}_prof_$cfg" -o run -- python3 "$R/bench.py" --config $cfg --no-sub --steps 10 --warmup 2 --no-cpu > "$OUT/${TAG}_prof_$cfg.log" 2>&1)
    rc=$?; echo "prof $cfg rc=$rc" >> "$OUT/${TAG}_status.txt"; fatal $rc prof_$cfg
  done
fi
echo "done $(date)" >> "$OUT/${TAG}_status.txt"
# PMC passes (separate runs, kernel-trace only): HBM traffic per kernel
if [ "${PMC:-0}" == "1" ]; then
  for cfg in ${PROF_CFGS:-c5}; do
    for ctr in FETCH_SIZE WRITE_SIZE; do
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d "$OUT/${TAG}_pmc_${cfg}_$ctr" -o run -- python3 "$R/bench.py" --config $cfg --no-sub --steps 3 --warmup 1 --no-cpu > "$OUT/${TAG}_pmc_${cfg}_$ctr.log" 2>&1)
      rc=$?; echo "pmc $cfg $ctr rc=$rc" >> "$OUT/${TAG}_status.txt"; fatal $rc pmc_$cfg
    done
  done
fi
echo "all done $(date)" >> "$OUT/${TAG}_status.txt"
