set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_fullsize.py tests/test_frontend.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/rows_tests.log 2>&1 || { echo tests failed; exit 1; }
for v in 0 1 0 1; do
  SDRGPU_TUNING=1 SDRGPU_FIR_ROWS=$v timeout -k 10 200 python bench.py --config c5 --steps 20 --warmup 3 --no-cpu >> gpurun_out/rows_ab.log 2>&1 || exit 1
done
