cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "onepass" -x -v --timeout 200 --timeout-method thread > gpurun_out/r5e_t.log 2>&1
echo "tests rc=$?" >> gpurun_out/r5e_t.log
AB_VAR=SDRGPU_FFT_1P AB_VALUES="0 1" AB_RUNS=2 bash tools/session.sh r5e ab
export SDRGPU_TUNING=1 SDRGPU_FFT_1P=1 SDRGPU_LIB_PATH=$GRAFT_REPO_ROOT/sdrpp_amd/lib_t1p/libsdrgpu.so
timeout -k 10 200 python tools/onepass_phases.py > gpurun_out/r5e_phases_vfo.json 2> gpurun_out/r5e_phases.err && \
timeout -k 10 200 python tools/onepass_phases.py --novfo > gpurun_out/r5e_phases_novfo.json 2>> gpurun_out/r5e_phases.err
