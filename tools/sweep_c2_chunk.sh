#!/bin/bash
# C2 (1M spectrum) step time vs the pass-A/B chunk size (SDRGPU_FFT_CHUNK_MB, tuning gate on), 2 interleaved rounds
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; OUT=$R/gpurun_out
for rep in 1 2; do for mb in 128 32 64 256; do
  env SDRGPU_TUNING=1 SDRGPU_FFT_CHUNK_MB=$mb timeout -k 10 200 python bench.py --config c2 --steps 20 --warmup 3 --no-cpu --no-sub >> $OUT/s4j_c2_$mb.jsonl 2>>$OUT/s4j_err.log || exit 1
done; done
