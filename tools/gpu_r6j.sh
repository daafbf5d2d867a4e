# r6j: phase stamps of ablation builds (wrong results, timing only): fp32 stage-1 twiddles (a8), + fp32 W_128 product (a40)
set -o pipefail
R=$PWD; OUT=gpurun_out
for v in a8 a40 t1p; do
  SDRGPU_LIB_PATH=$R/sdrpp_amd/lib_$v/libsdrgpu.so timeout -k 10 300 python tools/onepass_phases.py > $OUT/r6j_phases_$v.json 2>> $OUT/r6j_phases.err || exit $?
done
