# r6g: one-pass kernel with the ring's first row sets issued before the VFO half (lib_edma) vs tree:
# bits, interleaved C5 A/B, phase stamps of both (lib_t1p, lib_t1pe)
set -o pipefail
R=$PWD; OUT=gpurun_out
timeout -k 10 300 python tools/bits_digest.py > $OUT/r6g_bits_tree.json 2> $OUT/r6g_bits.err || exit $?
SDRGPU_LIB_PATH=$R/sdrpp_amd/lib_edma/libsdrgpu.so timeout -k 10 300 python tools/bits_digest.py > $OUT/r6g_bits_edma.json 2>> $OUT/r6g_bits.err || exit $?
AB_LIBS=edma AB_CFG=c5 AB_RUNS=3 bash tools/session.sh r6g ablib || exit $?
for v in t1p t1pe; do
  SDRGPU_LIB_PATH=$R/sdrpp_amd/lib_$v/libsdrgpu.so timeout -k 10 300 python tools/onepass_phases.py > $OUT/r6g_phases_$v.json 2>> $OUT/r6g_phases.err || exit $?
done
