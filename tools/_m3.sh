#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; OUT=$R/gpurun_out; mkdir -p $OUT
SDRGPU_FFT_CHUNK_MB=16 timeout -k 10 600 python -m pytest tests/test_gpu_parity.py tests/test_frontend.py -m gpu -q -x -p no:cacheprovider > $OUT/m3_tests.log 2>&1 || { echo "tests rc=$?" >> $OUT/m3_tests.log; exit 1; }
TAG=m3 CFG=c2 bash tools/sweep.sh "" "SDRGPU_FFT_MERGE=0" "SDRGPU_FFT_CHUNK_MB=128" "SDRGPU_FFT_MERGE=0 SDRGPU_FFT_CHUNK_MB=128" || exit 1
TAG=m3 CFG=c5 bash tools/sweep.sh "SDRGPU_FFT_CHUNK_MB=128" "SDRGPU_FFT_CHUNK_MB=192" "SDRGPU_FFT_CHUNK_MB=256" "" "SDRGPU_FFT_CHUNK_MB=128"
