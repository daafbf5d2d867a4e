cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider -rA > gpurun_out/g1_tests.log 2>&1; echo "rc=$?" >> gpurun_out/g1_tests.log
