# r6v: tail and fold workgroups interleaved in the tail+fold launch (lib_mix) vs tail first (tree): bits, C5 A/B
set -o pipefail
R=$PWD; OUT=gpurun_out
SDRGPU_LIB_PATH=$R/sdrpp_amd/lib_mix/libsdrgpu.so timeout -k 10 300 python tools/bits_digest.py > $OUT/r6v_bits_mix.json 2> $OUT/r6v_bits.err || exit $?
AB_LIBS=mix AB_CFG=c5 AB_RUNS=3 bash tools/session.sh r6v ablib || exit $?
