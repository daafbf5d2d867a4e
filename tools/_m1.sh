#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; OUT=$R/gpurun_out; mkdir -p $OUT
SDRGPU_FFT_MERGE=1 SDRGPU_FFT_CHUNK_MB=8 timeout -k 10 600 python -m pytest tests/test_gpu_parity.py tests/test_frontend.py -m gpu -q -x -p no:cacheprovider > $OUT/m1_tests.log 2>&1 || { echo "tests rc=$?" >> $OUT/m1_tests.log; exit 1; }
TAG=m1 CFG=c5 bash tools/sweep.sh "" "SDRGPU_FFT_MERGE=1" "" "SDRGPU_FFT_MERGE=1" "SDRGPU_FFT_MERGE=1 SDRGPU_FFT_CHUNK_MB=48" "SDRGPU_FFT_MERGE=1 SDRGPU_FFT_CHUNK_MB=32"
