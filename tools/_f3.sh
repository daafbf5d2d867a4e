cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 300 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/f4_tests.log 2>&1 ; echo "tests rc=$?" >> gpurun_out/f4_tests.log; \
TAG=f4 bash tools/ab.sh r0
