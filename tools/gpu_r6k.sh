# r6k: scheduling barriers beside the one-pass transform's workgroup barriers (lib_sb) vs tree: bits, C5 A/B, stamps
set -o pipefail
R=$PWD; OUT=gpurun_out
SDRGPU_LIB_PATH=$R/sdrpp_amd/lib_sb/libsdrgpu.so timeout -k 10 300 python tools/bits_digest.py > $OUT/r6k_bits_sb.json 2> $OUT/r6k_bits.err || exit $?
AB_LIBS=sb AB_CFG=c5 AB_RUNS=3 bash tools/session.sh r6k ablib || exit $?
SDRGPU_LIB_PATH=$R/sdrpp_amd/lib_t1psb/libsdrgpu.so timeout -k 10 300 python tools/onepass_phases.py > $OUT/r6k_phases_t1psb.json 2> $OUT/r6k_phases.err || exit $?
