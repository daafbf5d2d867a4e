cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
TAG=f8 CFG=c3 bash tools/sweep.sh "" "SDRGPU_FIR_K=8 SDRGPU_FIR_NT=128" "SDRGPU_FIR_K=8 SDRGPU_FIR_LDS_KB=150" "SDRGPU_FIR_K=2" "SDRGPU_FIR_K=4 SDRGPU_FIR_NT=128" && \
bash tools/pmc_sets.sh f8pmc "fir_kernel" $GRAFT_REPO_ROOT/bench.py --config c3 --steps 3 --warmup 1 --no-cpu
