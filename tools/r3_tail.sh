#!/bin/bash
# Round-3 per-call iteration: VFO / frontend / WFM / C5 tests, per-call timing, C5 bench A/B of
# the tail-chain build (stage 2 on the VALU FIR for large calls) vs SDRGPU_VFO_TAIL=0.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; OUT=$R/gpurun_out; TAG=${1:-tail}; mkdir -p $OUT
st() { echo "$1 rc=$2 $(date +%T)" >> $OUT/${TAG}_status.txt; case "$2" in 0) ;; *) exit "$2";; esac; }
echo "start $(date +%T)" > $OUT/${TAG}_status.txt
timeout -k 10 400 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  -k "vfo or VFO or frontend or wfm or c5 or stream or dropin" > $OUT/${TAG}_tests.log 2>&1
echo "tests rc=$? $(date +%T)" >> $OUT/${TAG}_status.txt
for rep in 1 2; do
  timeout -k 10 300 python tools/per_call.py 300 single > $OUT/${TAG}_pc_$rep.json 2>&1; st pc$rep $?
  SDRGPU_TUNING=1 SDRGPU_VFO_TAIL=0 timeout -k 10 300 python tools/per_call.py 300 single > $OUT/${TAG}_pc0_$rep.json 2>&1; st pc0$rep $?
done
for rep in 1 2; do
  timeout -k 10 300 python bench.py --config c5 --steps 20 --no-cpu --no-sub > $OUT/${TAG}_c5_$rep.json 2>&1; st c5$rep $?
  SDRGPU_TUNING=1 SDRGPU_VFO_TAIL=0 timeout -k 10 300 python bench.py --config c5 --steps 20 --no-cpu --no-sub > $OUT/${TAG}_c50_$rep.json 2>&1; st c50$rep $?
done
echo "all done $(date +%T)" >> $OUT/${TAG}_status.txt
