# r5j: packed-fp32 VFO segment (bits + speed vs the scalar build), late VFO placements (+ traffic)
set -o pipefail
OUT=gpurun_out
for v in tree pk0; do
  L=$PWD/sdrpp_amd/lib/libsdrgpu.so; [ "$v" = tree ] || L=$PWD/sdrpp_amd/lib_$v/libsdrgpu.so
  SDRGPU_LIB_PATH=$L timeout -k 10 300 python tools/bits_digest.py > $OUT/r5j_bits_$v.json 2> $OUT/r5j_bits_$v.err || exit $?
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "vfo or rxvfo or onepass or tail or rows or frontend or fir" -q \
  -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/r5j_tests.log 2>&1; [ $? -le 1 ] || exit 9
AB_LIBS="pk0 late1 late2" AB_RUNS=2 bash tools/session.sh r5j ablib || exit $?
for v in late1 late2; do
  SDRGPU_LIB_PATH=$PWD/sdrpp_amd/lib_$v/libsdrgpu.so PMC_CFGS=c5 bash tools/session.sh r5j_$v pmc || exit $?
done
