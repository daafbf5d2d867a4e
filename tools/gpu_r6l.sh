# r6l: stamps inside quarter r0's stage-1 finish (with scheduling barriers around every stamp: lib_t1psb; without: lib_t1p)
set -o pipefail
R=$PWD; OUT=gpurun_out
for v in t1psb t1p; do
  SDRGPU_LIB_PATH=$R/sdrpp_amd/lib_$v/libsdrgpu.so timeout -k 10 300 python tools/onepass_phases.py > $OUT/r6l_phases_$v.json 2>> $OUT/r6l_phases.err || exit $?
done
