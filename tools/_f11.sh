cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/f11_tests.log 2>&1; echo "rc=$?" >> gpurun_out/f11_tests.log; \
SDRGPU_CHAN_TWO=1 timeout -k 10 300 python -m pytest tests/test_channelizer.py -q -p no:cacheprovider > gpurun_out/f11_chan2_tests.log 2>&1; echo "rc=$?" >> gpurun_out/f11_chan2_tests.log; \
TAG=f11 CFGS="c5 c2" bash tools/ab.sh r2 && \
TAG=f11 CFG=c5 bash tools/sweep.sh "SDRGPU_FFT_PIPE=0" "SDRGPU_FFT_CHUNK_MB=32" "SDRGPU_FFT_CHUNK_MB=128" && \
TAG=f11 CFG=c4 bash tools/sweep.sh "" "SDRGPU_CHAN_TWO=1" "SDRGPU_CHAN_TWO=1 SDRGPU_CHAN_FPW=512"
