# r6f: 1M pass B at sequence stride 1090 (tree) vs 1089 (lib_pb1089): GPU tests, interleaved C2 A/B, SQ LDS counters
set -o pipefail
R=$PWD; OUT=gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/r6f_tests.log 2>&1; [ $? -le 1 ] || exit 9
AB_LIBS=pb1089 AB_CFG=c2 AB_RUNS=3 bash tools/session.sh r6f ablib || exit $?
bash tools/pmc_sets.sh r6f_sq_c2 "fft_pass[AB]_1m_kernel" "$R/bench.py" --config c2 --no-sub --no-cpu --no-ulp --steps 3 --warmup 1 || exit $?
