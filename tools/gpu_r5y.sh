# r5y: one-pass twiddle products in fp64 (SDRGPU_1P_TW64 builds): near-peak ulps (AES17 / tones / corpus) and C5 time
set -o pipefail
OUT=gpurun_out
for v in tw2 tw8; do
  L=$PWD/sdrpp_amd/lib/libsdrgpu.so; [ "$v" = tree ] || L=$PWD/sdrpp_amd/lib_$v/libsdrgpu.so
  SDRGPU_LIB_PATH=$L SDRGPU_REPORT_DIR=$OUT/r5y_rep_$v timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py \
    -k "ulp_distribution or ulp_corpus or f64_within" -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/r5y_tests_$v.log 2>&1
  [ $? -le 1 ] || exit 9
done
AB_LIBS="tw2 tw8 tw3" AB_RUNS=2 bash tools/session.sh r5y ablib || exit $?
