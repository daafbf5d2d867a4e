# r5n: VFO tail kernel at 8 outputs per thread with packed MACs (bits, parity, C5 step vs the r5k build),
# the WFM FIR's register window (SDRGPU_FIR_K), per-kernel C5 trace
set -o pipefail
OUT=gpurun_out
timeout -k 10 300 python tools/bits_digest.py > $OUT/r5n_bits_tree.json 2> $OUT/r5n_bits_tree.err || exit $?
timeout -k 10 900 python -u -m pytest tests -k "tail or vfo or wfm or fir or broadcast or frontend or stereo" -q -m gpu \
  -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/r5n_tests.log 2>&1; [ $? -le 1 ] || exit 9


PROF_CFGS=c5 bash tools/session.sh r5n prof || exit $?
