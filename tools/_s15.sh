cd $GRAFT_REPO_ROOT && BENCH_CFGS="c5 c3 c4 c2" PROF_CFGS="c5 c3 c4 c2" CPUSEC=10 bash tools/gpu_session.sh s15 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/s15_smoke.log 2>&1
