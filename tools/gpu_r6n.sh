# r6n: BroadcastFM big calls with packed FMAs (tree) vs the scalar chains (lib_wfmold): GPU tests, bits, C5 A/B
set -o pipefail
R=$PWD; OUT=gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/r6n_tests.log 2>&1; [ $? -le 1 ] || exit 9
timeout -k 10 300 python tools/bits_digest.py > $OUT/r6n_bits_tree.json 2> $OUT/r6n_bits.err || exit $?
SDRGPU_LIB_PATH=$R/sdrpp_amd/lib_wfmold/libsdrgpu.so timeout -k 10 300 python tools/bits_digest.py > $OUT/r6n_bits_wfmold.json 2>> $OUT/r6n_bits.err || exit $?
AB_LIBS=wfmold AB_CFG=c5 AB_RUNS=3 bash tools/session.sh r6n ablib || exit $?
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/r6n_prof -o run -- python3 $R/bench.py --config c5 --no-sub --no-cpu --no-ulp --steps 10 --warmup 2 > $R/$OUT/r6n_prof.json 2> $R/$OUT/r6n_prof.err || exit $?
