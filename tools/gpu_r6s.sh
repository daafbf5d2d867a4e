# r6s: 1M chunks alternating between two streams (SDRGPU_FFT_2S=1) vs one: chunking bit-identity tests, C2 A/B
set -o pipefail
R=$PWD; OUT=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -k "chunking or 1m or c2" -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/r6s_tests.log 2>&1 || exit 9
AB_VAR=SDRGPU_FFT_2S AB_VALUES="0 1" AB_CFG=c2 AB_RUNS=3 bash tools/session.sh r6s ab || exit $?
