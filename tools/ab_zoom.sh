#!/bin/bash
# A/B on one box: the C5 step with and without the fused waterfall zoom rows (interleaved)
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; OUT=$R/gpurun_out; mkdir -p $OUT; TAG=${1:-abz}
for k in 1 2 3; do
  for z in 1 0; do
    BENCH_C5_ZOOM=$z timeout -k 10 200 python bench.py --config c5 --no-sub --no-cpu --steps 20 --warmup 3 >> $OUT/${TAG}_zoom$z.jsonl 2>>$OUT/${TAG}_err.log || exit 1
  done
done
