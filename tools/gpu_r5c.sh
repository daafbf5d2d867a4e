cd $GRAFT_REPO_ROOT
export SDRGPU_TUNING=1 SDRGPU_FFT_1P=1 SDRGPU_LIB_PATH=$GRAFT_REPO_ROOT/sdrpp_amd/lib_t1p/libsdrgpu.so
timeout -k 10 200 python tools/onepass_phases.py > gpurun_out/r5c_phases_vfo.json 2> gpurun_out/r5c_phases.err && \
timeout -k 10 200 python tools/onepass_phases.py --novfo > gpurun_out/r5c_phases_novfo.json 2>> gpurun_out/r5c_phases.err
