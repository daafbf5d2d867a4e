cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "onepass or vfo_fused or zoom_rows" -x -v --timeout 200 --timeout-method thread > gpurun_out/r5b_t.log 2>&1
echo "tests rc=$?" >> gpurun_out/r5b_t.log
AB_VAR=SDRGPU_FFT_1P AB_VALUES="0 1" AB_RUNS=2 bash tools/session.sh r5b ab
