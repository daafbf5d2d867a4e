cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "onepass or zoom" -x -q --timeout 200 --timeout-method thread > gpurun_out/r5f_t.log 2>&1
echo "tests rc=$?" >> gpurun_out/r5f_t.log
export SDRGPU_TUNING=1 SDRGPU_FFT_1P=1
AB_LIBS="nodma" AB_RUNS=2 bash tools/session.sh r5f ablib
PMC_CFGS=c5 bash tools/session.sh r5f pmc
bash tools/pmc_sets.sh r5f_sq fft_1p_kernel $R/bench.py --config c5 --no-sub --no-cpu --no-ulp --steps 3 --warmup 1
