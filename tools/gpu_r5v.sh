# r5v: streaming tail with compile-time stage loops: bits, parity, A/B (no-arithmetic ablation, old tail), trace
set -o pipefail
OUT=gpurun_out
timeout -k 10 300 python tools/bits_digest.py > $OUT/r5v_bits_tree.json 2> $OUT/r5v_bits_tree.err || exit $?
timeout -k 10 900 python -u -m pytest tests -k "tail or vfo or rxvfo or decim" -q -m gpu \
  -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/r5v_tests.log 2>&1; [ $? -le 1 ] || exit 9
AB_LIBS="sabl1" AB_RUNS=2 bash tools/session.sh r5v ablib || exit $?
AB_VAR=SDRGPU_TAIL_STREAM AB_VALUES="0 1" AB_RUNS=2 bash tools/session.sh r5v_s ab || exit $?
PROF_CFGS=c5 bash tools/session.sh r5v prof || exit $?
