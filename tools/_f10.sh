cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider -k "fft or spectrum or smoke or dropin" > gpurun_out/f10_tests.log 2>&1; echo "rc=$?" >> gpurun_out/f10_tests.log; \
TAG=f10 CFGS="c5 c2" bash tools/ab.sh r2 && \
TAG=f10 CFG=c5 bash tools/sweep.sh "SDRGPU_FFT_PIPE=0" "SDRGPU_FFT_CHUNK_MB=32" "SDRGPU_FFT_CHUNK_MB=128"
