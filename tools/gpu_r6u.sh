# r6u: the big-call VFO tail at 2 outputs per thread (lib_tk2) vs 4 (tree), now that it shares its launch with the zoom fold
set -o pipefail
R=$PWD; OUT=gpurun_out
SDRGPU_LIB_PATH=$R/sdrpp_amd/lib_tk2/libsdrgpu.so timeout -k 10 300 python tools/bits_digest.py > $OUT/r6u_bits_tk2.json 2> $OUT/r6u_bits.err || exit $?
AB_LIBS=tk2 AB_CFG=c5 AB_RUNS=3 bash tools/session.sh r6u ablib || exit $?
