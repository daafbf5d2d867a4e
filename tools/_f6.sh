cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
TAG=f6 CFG=c3 bash tools/sweep.sh "" "SDRGPU_FIR_NT=128" "SDRGPU_FIR_NT=64" "SDRGPU_FIR_LDS_KB=40" "SDRGPU_FIR_TPW=2" "SDRGPU_LIB_PATH=$GRAFT_REPO_ROOT/abtest/libsdrgpu_r0.so" && \
TAG=f6 CFG=c5 bash tools/sweep.sh "" "SDRGPU_FFT_SA2=0" "SDRGPU_FFT_SA2=64" "SDRGPU_FIR_NT=128" "SDRGPU_LIB_PATH=$GRAFT_REPO_ROOT/abtest/libsdrgpu_r0.so"
