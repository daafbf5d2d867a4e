#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; OUT=$R/gpurun_out; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_frontend.py tests/test_loops.py -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/m5_tests.log 2>&1 || { echo "tests rc=$?" >> $OUT/m5_tests.log; exit 1; }
SDRGPU_FIR_MFMA=2 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "fir or ddc or rxvfo or power or wfm or fm" > $OUT/m5_tests2.log 2>&1; echo "rc=$?" >> $OUT/m5_tests2.log
TAG=m5 CFG=c3 bash tools/sweep.sh "SDRGPU_FIR_MFMA=0" "" "SDRGPU_FIR_MFMA=0" "" || exit 1
TAG=m5 CFG=c5 bash tools/sweep.sh "SDRGPU_FIR_MFMA=0" "" "SDRGPU_FIR_MFMA=2"
