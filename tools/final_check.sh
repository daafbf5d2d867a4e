#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; OUT=$R/gpurun_out; mkdir -p $OUT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/final_smoke.log 2>&1 || { echo "smoke rc=$?" >> $OUT/f_smoke.log; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/final_tests.log 2>&1 || { echo "tests rc=$?" >> $OUT/final_tests.log; exit 1; }
timeout -k 10 400 python bench.py > $OUT/final_bench.json 2> $OUT/final_bench.err
