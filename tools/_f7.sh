cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/f7_tests.log 2>&1; echo "rc=$?" >> gpurun_out/f7_tests.log; \
TAG=f7 CFGS="c3 c5" bash tools/ab.sh r1
