cd $GRAFT_REPO_ROOT && mkdir -p gurpun_out gpurun_out && \
timeout -k 10 300 python -m pytest tests -m gpu -q -k "fft or spectrum or smoke" -p no:cacheprovider > gpurun_out/a2_tests.log 2>&1 ; echo "tests rc=$?" >> gpurun_out/a2_tests.log; \
timeout -k 10 600 python tools/fft_variants.py '[{"SDRGPU_FFT_SA2":0},{"SDRGPU_FFT_SA2":16},{"SDRGPU_FFT_SA2":32},{"SDRGPU_FFT_SA2":64}]' > gpurun_out/a2_var.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/a2_prof -o run -- python3 $GRAFT_REPO_ROOT/tools/fft_one.py 65536 65536 4096 10 > $GRAFT_REPO_ROOT/gpurun_out/a2_prof.log 2>&1
