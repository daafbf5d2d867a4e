# r5l: the VFO's stage-1 half from the one-pass kernel's L2-hit segment batches (bits, parity, speed vs the previous build, traffic)
set -o pipefail
OUT=gpurun_out
timeout -k 10 300 python tools/bits_digest.py > $OUT/r5l_bits_tree.json 2> $OUT/r5l_bits_tree.err || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "vfo or onepass or zoom" -q \
  -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/r5l_tests.log 2>&1; [ $? -le 1 ] || exit 9
AB_LIBS="old" AB_RUNS=3 bash tools/session.sh r5l ablib || exit $?
PMC_CFGS=c5 bash tools/session.sh r5l pmc || exit $?
