set -o pipefail
R=$PWD
bash tools/session.sh r7b ulpcorpus || exit $?
SDRGPU_LIB_PATH=$R/sdrpp_amd/lib_tw1/libsdrgpu.so bash tools/session.sh r7b_tw1 ulpcorpus || exit $?
SDRGPU_LIB_PATH=$R/sdrpp_amd/lib_tw3/libsdrgpu.so bash tools/session.sh r7b_tw3 ulpcorpus || exit $?
AB_LIBS="tw1 tw3" AB_CFG=c5 AB_RUNS=3 bash tools/session.sh r7b_c5 ablib || exit $?
AB_LIBS="tw3" AB_CFG=c2 AB_RUNS=2 bash tools/session.sh r7b_c2 ablib || exit $?
