#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; OUT=$R/gpurun_out; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread -k "fir or ddc or rxvfo or power or wfm or fm" > $OUT/m6_tests.log 2>&1 || { echo "tests rc=$?" >> $OUT/m6_tests.log; exit 1; }
SDRGPU_FIR_MFMA=2 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread -k "fir or ddc or rxvfo or power or wfm or fm" > $OUT/m6_tests2.log 2>&1 || { echo "tests rc=$?" >> $OUT/m6_tests2.log; exit 1; }
TAG=m6 CFG=c3 bash tools/sweep.sh "SDRGPU_FIR_MFMA_NW=4" "" "SDRGPU_FIR_MFMA_NW=4" "" "SDRGPU_FIR_MFMA=0"
