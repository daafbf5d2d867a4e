#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; OUT=$R/gpurun_out; mkdir -p $OUT
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -m gpu -q -x -p no:cacheprovider -k "merged or fft" > $OUT/m2_tests.log 2>&1 || { echo "tests rc=$?" >> $OUT/m2_tests.log; exit 1; }
TAG=m2 CFG=c5 bash tools/sweep.sh "" "SDRGPU_FFT_CHUNK_MB=80" "SDRGPU_FFT_CHUNK_MB=96" "SDRGPU_FFT_CHUNK_MB=128" "SDRGPU_FFT_MERGE=0" ""
