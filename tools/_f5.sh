cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
for gm in 1 4 16 64; do SDRGPU_FIR_GRID_MUL=$gm timeout -k 10 300 python bench.py --config c3 --steps 20 --no-cpu > gpurun_out/f5_c3_gm$gm.json 2>&1 || exit $?; done; \
SDRGPU_LIB_PATH=$GRAFT_REPO_ROOT/abtest/libsdrgpu_r0.so timeout -k 10 300 python bench.py --config c3 --steps 20 --no-cpu > gpurun_out/f5_c3_r0.json 2>&1
