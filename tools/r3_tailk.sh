#!/bin/bash
# fir_tail_kernel variants (sdrpp_amd/lib_<v>): the tail tests, then a per-call kernel trace each
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; OUT=$R/gpurun_out; TAG=${1:-tk}; mkdir -p $OUT
st() { echo "$1 rc=$2 $(date +%T)" >> $OUT/${TAG}_status.txt; case "$2" in 0) ;; *) exit "$2";; esac; }
echo "start $(date +%T)" > $OUT/${TAG}_status.txt
for v in ${VARS:-k2p0 k1p0 k2p1}; do
  L=$R/sdrpp_amd/lib_$v/libsdrgpu.so
  SDRGPU_LIB_PATH=$L timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider -k "tail or rxvfo" --timeout 120 --timeout-method thread > $OUT/${TAG}_${v}_tests.log 2>&1
  st tests_$v $?
  (cd /tmp && export TMPDIR=/tmp && SDRGPU_LIB_PATH=$L timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/${TAG}_$v -o run -- python3 $R/tools/per_call.py 60 single > $OUT/${TAG}_$v.log 2>&1)
  st pct_$v $?
done
echo "all done $(date +%T)" >> $OUT/${TAG}_status.txt
