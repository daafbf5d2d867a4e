cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 300 python -m pytest tests/test_channelizer.py -q -p no:cacheprovider > gpurun_out/c4_tests.log 2>&1; echo "rc=$?" >> gpurun_out/c4_tests.log; \
timeout -k 10 300 python bench.py --config c4 --steps 20 --no-cpu > gpurun_out/c4_bench.json 2>&1 && \
SDRGPU_CHAN_FPW=128 timeout -k 10 300 python bench.py --config c4 --steps 20 --no-cpu > gpurun_out/c4_bench_f128.json 2>&1 && \
SDRGPU_CHAN_FPW=512 timeout -k 10 300 python bench.py --config c4 --steps 20 --no-cpu > gpurun_out/c4_bench_f512.json 2>&1
