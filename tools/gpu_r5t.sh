# r5t: fused big-call WFM (bits, parity), the VFO tail kernel's big-call shape A/B, per-kernel C5 trace
set -o pipefail
OUT=gpurun_out
timeout -k 10 300 python tools/bits_digest.py > $OUT/r5t_bits_tree.json 2> $OUT/r5t_bits_tree.err || exit $?
timeout -k 10 900 python -u -m pytest tests -k "tail or vfo or rxvfo or decim or wfm or fm" -q -m gpu \
  -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/r5t_tests.log 2>&1; [ $? -le 1 ] || exit 9

PROF_CFGS=c5 bash tools/session.sh r5t prof || exit $?
