# r6d: one-pass above 64 frames only: GPU tests, C5 bench line with the per-call figures
set -o pipefail
OUT=gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/r6d_tests.log 2>&1; [ $? -le 1 ] || exit 9
timeout -k 10 600 python bench.py --config c5 --no-cpu --no-ulp > $OUT/r6d_bench.json 2> $OUT/r6d_bench.err || exit $?
