# r6p: the zoom fold in the VFO tail's launch (tree) vs its own launch (lib_prefold): GPU tests, bits, C5 A/B, kernel trace
set -o pipefail
R=$PWD; OUT=gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/r6p_tests.log 2>&1; [ $? -le 1 ] || exit 9
timeout -k 10 300 python tools/bits_digest.py > $OUT/r6p_bits_tree.json 2> $OUT/r6p_bits.err || exit $?
SDRGPU_LIB_PATH=$R/sdrpp_amd/lib_prefold/libsdrgpu.so timeout -k 10 300 python tools/bits_digest.py > $OUT/r6p_bits_prefold.json 2>> $OUT/r6p_bits.err || exit $?
AB_LIBS=prefold AB_CFG=c5 AB_RUNS=3 bash tools/session.sh r6p ablib || exit $?
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/r6p_prof -o run -- python3 $R/bench.py --config c5 --no-sub --no-cpu --no-ulp --steps 10 --warmup 2 > $R/$OUT/r6p_prof.json 2> $R/$OUT/r6p_prof.err || exit $?
