cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 600 python -m pytest tests/test_loops.py tests/test_channelizer.py -q -p no:cacheprovider > gpurun_out/l4_tests.log 2>&1; echo "rc=$?" >> gpurun_out/l4_tests.log
