# r7h: fp64 64k pass B at 32 rows per workgroup (tree) vs 16 (lib_sb16): f64 tests + cost, interleaved
set -o pipefail
R=$PWD
PYTEST_K="f64" bash tools/session.sh r7h testk || exit $?
for k in 1 2; do
  timeout -k 10 300 python tools/f64_cost.py >> gpurun_out/r7h_f64cost_tree.json 2>> gpurun_out/r7h_f64cost.err || exit $?
  SDRGPU_LIB_PATH=$R/sdrpp_amd/lib_sb16/libsdrgpu.so timeout -k 10 300 python tools/f64_cost.py >> gpurun_out/r7h_f64cost_sb16.json 2>> gpurun_out/r7h_f64cost.err || exit $?
done
