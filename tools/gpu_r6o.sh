# r6o: BroadcastFM big calls at 4 outputs per thread (lib_wfm4) vs 8 (tree): WFM tests + bits on the variant, C5 A/B
set -o pipefail
R=$PWD; OUT=gpurun_out
SDRGPU_LIB_PATH=$R/sdrpp_amd/lib_wfm4/libsdrgpu.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -k "wfm or fm" -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/r6o_tests.log 2>&1 || exit 9
SDRGPU_LIB_PATH=$R/sdrpp_amd/lib_wfm4/libsdrgpu.so timeout -k 10 300 python tools/bits_digest.py > $OUT/r6o_bits_wfm4.json 2> $OUT/r6o_bits.err || exit $?
AB_LIBS=wfm4 AB_CFG=c5 AB_RUNS=3 bash tools/session.sh r6o ablib || exit $?
cd /tmp && export TMPDIR=/tmp && SDRGPU_LIB_PATH=$R/sdrpp_amd/lib_wfm4/libsdrgpu.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/r6o_prof -o run -- python3 $R/bench.py --config c5 --no-sub --no-cpu --no-ulp --steps 10 --warmup 2 > $R/$OUT/r6o_prof.json 2> $R/$OUT/r6o_prof.err || exit $?
