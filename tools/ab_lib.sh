#!/bin/bash
# A/B of two builds of libsdrgpu on one box (interleaved): sdrpp_amd/lib_old vs sdrpp_amd/lib,
# bench config $2 (default c5), 3 rounds
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; OUT=$R/gpurun_out; mkdir -p $OUT; TAG=${1:-ablib}; CFG=${2:-c5}
for k in 1 2 3; do
  for v in old new; do
    if [ $v == old ]; then L=$R/sdrpp_amd/lib_old/libsdrgpu.so; else L=$R/sdrpp_amd/lib/libsdrgpu.so; fi
    SDRGPU_LIB_PATH=$L timeout -k 10 200 python bench.py --config $CFG --no-sub --no-cpu --steps 20 --warmup 3 >> $OUT/${TAG}_$v.jsonl 2>>$OUT/${TAG}_err.log || exit 1
  done
done
