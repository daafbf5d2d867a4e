# r6q: the one-pass kernel's VFO half with both segments unrolled (lib_vfou) vs tree: bits, C5 A/B
set -o pipefail
R=$PWD; OUT=gpurun_out
SDRGPU_LIB_PATH=$R/sdrpp_amd/lib_vfou/libsdrgpu.so timeout -k 10 300 python tools/bits_digest.py > $OUT/r6q_bits_vfou.json 2> $OUT/r6q_bits.err || exit $?
AB_LIBS=vfou AB_CFG=c5 AB_RUNS=3 bash tools/session.sh r6q ablib || exit $?
