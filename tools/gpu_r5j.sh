set -o pipefail
AB_LIBS="late1 late2" AB_RUNS=2 bash tools/session.sh r5j ablib || exit $?
for v in late1 late2; do
  SDRGPU_LIB_PATH=$PWD/sdrpp_amd/lib_$v/libsdrgpu.so PMC_CFGS=c5 bash tools/session.sh r5j_$v pmc || exit $?
done
