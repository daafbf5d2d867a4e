cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "onepass or zoom" -x -q --timeout 200 --timeout-method thread > gpurun_out/r5g_t.log 2>&1
echo "tests rc=$?" >> gpurun_out/r5g_t.log
export SDRGPU_TUNING=1 SDRGPU_FFT_1P=1
AB_LIBS="vfou" AB_RUNS=3 bash tools/session.sh r5g ablib
