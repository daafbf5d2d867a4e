# r5u: streaming tail plan (debug print) and an ablation build without the stage arithmetic
set -o pipefail
OUT=gpurun_out
SDRGPU_TUNING=1 SDRGPU_TAIL_DEBUG=1 timeout -k 10 300 python bench.py --config c5 --no-sub --no-cpu --no-ulp --steps 3 --warmup 1 > $OUT/r5u_dbg.json 2> $OUT/r5u_dbg.err || exit $?
AB_LIBS="sabl1" AB_RUNS=2 bash tools/session.sh r5u ablib || exit $?
