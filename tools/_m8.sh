#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; OUT=$R/gpurun_out; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_frontend.py -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/m8_tests.log 2>&1 || { echo "tests rc=$?" >> $OUT/m8_tests.log; exit 1; }
SDRGPU_FIR_MFMA_PS=2 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread -k "fir or ddc or rxvfo or power or wfm or fm" > $OUT/m8_tests2.log 2>&1 || { echo "tests rc=$?" >> $OUT/m8_tests2.log; exit 1; }
TAG=m8 CFG=c5 bash tools/sweep.sh "SDRGPU_FIR_MFMA_PS=0" "" "SDRGPU_FIR_MFMA_PS=0" "" || exit 1
TAG=m8 CFG=c3 bash tools/sweep.sh "" "SDRGPU_FIR_MFMA_PS=2"
