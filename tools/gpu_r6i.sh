# r6i: the stage-1 twiddle seeds loaded at the kernel start (lib_t64) vs tree: bits, C5 A/B, phase stamps
set -o pipefail
R=$PWD; OUT=gpurun_out
SDRGPU_LIB_PATH=$R/sdrpp_amd/lib_t64/libsdrgpu.so timeout -k 10 300 python tools/bits_digest.py > $OUT/r6i_bits_t64.json 2> $OUT/r6i_bits.err || exit $?
AB_LIBS=t64 AB_CFG=c5 AB_RUNS=3 bash tools/session.sh r6i ablib || exit $?
SDRGPU_LIB_PATH=$R/sdrpp_amd/lib_t1p64/libsdrgpu.so timeout -k 10 300 python tools/onepass_phases.py > $OUT/r6i_phases_t1p64.json 2> $OUT/r6i_phases.err || exit $?
