# r7b: the 16-wave one-pass kernel (lib_op16) correctness + C5 A/B; tail-stream correctness + A/B;
# fp64 twiddle-product accuracy variants (tonal corpus) + timing
set -o pipefail
R=$PWD
SDRGPU_LIB_PATH=$R/sdrpp_amd/lib_op16/libsdrgpu.so PYTEST_K="onepass or tail_stream or 64k_rows_vs_call_size or zoom_vfo or tonal_corpus or ulp_distribution" bash tools/session.sh r7b_op16 testk || exit $?
AB_LIBS="op16" AB_CFG=c5 AB_RUNS=3 bash tools/session.sh r7b_op16 ablib || exit $?
PYTEST_K="tail_stream or 64k_rows_vs_call_size or onepass or zoom_vfo" bash tools/session.sh r7b testk || exit $?
AB_VAR=BENCH_C5_TAIL AB_VALUES="0 1" AB_CFG=c5 AB_RUNS=2 bash tools/session.sh r7b_tail ab || exit $?
PYTEST_K="tonal_corpus or ulp_distribution" bash tools/session.sh r7b_tree testk || exit $?
SDRGPU_LIB_PATH=$R/sdrpp_amd/lib_tw1/libsdrgpu.so PYTEST_K="tonal_corpus or ulp_distribution" bash tools/session.sh r7b_tw1 testk || exit $?
SDRGPU_LIB_PATH=$R/sdrpp_amd/lib_tw3/libsdrgpu.so PYTEST_K="tonal_corpus or ulp_distribution" bash tools/session.sh r7b_tw3 testk || exit $?
AB_LIBS="tw1 tw3" AB_CFG=c5 AB_RUNS=2 bash tools/session.sh r7b_c5 ablib || exit $?
AB_LIBS="tw3" AB_CFG=c2 AB_RUNS=2 bash tools/session.sh r7b_c2 ablib || exit $?
