cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 300 python tools/fft_variants.py '[{}, {"SDRGPU_FFT_N1":64}, {"SDRGPU_FFT_N1":128}, {"SDRGPU_FFT_N1":512}, {"SDRGPU_FFT_N1":1024}, {"SDRGPU_FFT_N1":512,"SDRGPU_FFT_SA2":16}, {"SDRGPU_FFT_N1":1024,"SDRGPU_FFT_SA2":16}]' > gpurun_out/f12_var.log 2>&1
