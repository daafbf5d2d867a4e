cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "onepass" -x -v --timeout 200 --timeout-method thread > gpurun_out/r5e_t.log 2>&1
echo "tests rc=$?" >> gpurun_out/r5e_t.log
AB_VAR=SDRGPU_FFT_1P AB_VALUES="0 1" AB_RUNS=2 bash tools/session.sh r5e ab
SDRGPU_TUNING=1 SDRGPU_FFT_1P=1 AB_LIBS="nodma early" AB_RUNS=2 bash tools/session.sh r5e2 ablib
export SDRGPU_TUNING=1 SDRGPU_FFT_1P=1 SDRGPU_LIB_PATH=$GRAFT_REPO_ROOT/sdrpp_amd/lib_t1p/libsdrgpu.so
timeout -k 10 200 python tools/onepass_phases.py > gpurun_out/r5e_phases_vfo.json 2> gpurun_out/r5e_phases.err && \
timeout -k 10 200 python tools/onepass_phases.py --novfo > gpurun_out/r5e_phases_novfo.json 2>> gpurun_out/r5e_phases.err
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r5e_prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config c5 --no-sub --no-cpu --no-ulp --steps 5 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/r5e_prof.json 2> $GRAFT_REPO_ROOT/gpurun_out/r5e_prof.err
