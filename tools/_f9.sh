cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider -k "fir or FIR or vfo or ddc or wfm or fm or decim or resampl or am or ssb" > gpurun_out/f9_tests.log 2>&1; echo "rc=$?" >> gpurun_out/f9_tests.log; \
TAG=f9 CFGS="c3 c5" bash tools/ab.sh r2
