#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; OUT=$R/gpurun_out; mkdir -p $OUT
SDRGPU_FIR_MFMA_NW=4 bash tools/pmc_sets.sh m7 "fir_mfma" $R/bench.py --config c3 --steps 2 --warmup 1 --no-cpu --log2-batch 26
