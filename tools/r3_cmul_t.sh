#!/bin/bash
# packed-asm cmul: every -m gpu test, then the per-window error distribution (24 frames per case) for
# this build and the previous one (lib_old)
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; OUT=$R/gpurun_out; TAG=${1:-cmt}; mkdir -p $OUT
st() { echo "$1 rc=$2 $(date +%T)" >> $OUT/${TAG}_status.txt; case "$2" in 0) ;; *) exit "$2";; esac; }
echo "start $(date +%T)" > $OUT/${TAG}_status.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/${TAG}_tests.log 2>&1
st tests $?
FRAMES=24 timeout -k 10 400 python tools/fft_window_err.py > $OUT/${TAG}_we_new.json 2>>$OUT/${TAG}_we.err; st we_new $?
SDRGPU_LIB_PATH=$R/sdrpp_amd/lib_old/libsdrgpu.so FRAMES=24 timeout -k 10 400 python tools/fft_window_err.py > $OUT/${TAG}_we_old.json 2>>$OUT/${TAG}_we.err; st we_old $?
echo "all done $(date +%T)" >> $OUT/${TAG}_status.txt
