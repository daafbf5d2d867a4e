# r5z: W_128 twiddle in fp64 at the combine: accuracy (ulp tests), one-pass parity, bits, time vs HEAD~ (prev) and the in-transform form (tw2)
set -o pipefail
OUT=gpurun_out
SDRGPU_REPORT_DIR=$OUT/r5z_rep timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py \
  -k "ulp or f64_within or onepass or vfo or zoom" -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/r5z_tests.log 2>&1
[ $? -le 1 ] || exit 9
timeout -k 10 300 python tools/bits_digest.py > $OUT/r5z_bits_tree.json 2> $OUT/r5z_bits_tree.err || exit $?
AB_LIBS="prev tw2" AB_RUNS=3 bash tools/session.sh r5z ablib || exit $?
