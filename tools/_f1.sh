cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
SKIP_TESTS=0 BENCH_CFGS="c3 c5" STEPS=20 CPUSEC=2 PROF_CFGS="c3 c5" bash tools/gpu_session.sh f2 && \
SDRGPU_FIR_GRID_MUL=2 timeout -k 10 300 python bench.py --config c3 --steps 20 --no-cpu > gpurun_out/f2_c3_g2.json 2>&1 && \
SDRGPU_FIR_GRID_MUL=4 timeout -k 10 300 python bench.py --config c3 --steps 20 --no-cpu > gpurun_out/f2_c3_g4.json 2>&1
