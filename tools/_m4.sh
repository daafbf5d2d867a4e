#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; OUT=$R/gpurun_out; mkdir -p $OUT
timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider > $OUT/m4_tests.log 2>&1 || { echo "tests rc=$?" >> $OUT/m4_tests.log; exit 1; }
TAG=m4 CFG=c5 bash tools/sweep.sh "" "SDRGPU_FFT_MERGE=0" "" "SDRGPU_FFT_MERGE=0"
