# r6a: fp64-interior mode: fast log (default) vs libm log10, pass-A width 8 vs 16 (cost + exactness);
# then the combine-side fp64 W_128 session (r5z)
set -o pipefail
OUT=gpurun_out
for v in tree liblog sa8; do
  L=$PWD/sdrpp_amd/lib/libsdrgpu.so; [ "$v" = tree ] || L=$PWD/sdrpp_amd/lib_$v/libsdrgpu.so
  SDRGPU_LIB_PATH=$L timeout -k 10 300 python tools/f64_cost.py > $OUT/r6a_f64_$v.json 2> $OUT/r6a_f64_$v.err || exit $?
done
SDRGPU_REPORT_DIR=$OUT/r6a_rep timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "f64 or corpus" -q \
  -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/r6a_tests.log 2>&1; [ $? -le 1 ] || exit 9
bash tools/gpu_r5z.sh
