# r6h: one-pass phase stamps by transform stage (lib_t1p), early-DMA default
set -o pipefail
R=$PWD; OUT=gpurun_out
SDRGPU_LIB_PATH=$R/sdrpp_amd/lib_t1p/libsdrgpu.so timeout -k 10 300 python tools/onepass_phases.py > $OUT/r6h_phases_t1p.json 2> $OUT/r6h_phases.err || exit $?
SDRGPU_LIB_PATH=$R/sdrpp_amd/lib_t1p/libsdrgpu.so timeout -k 10 300 python tools/onepass_phases.py --novfo > $OUT/r6h_phases_t1p_novfo.json 2>> $OUT/r6h_phases.err || exit $?
