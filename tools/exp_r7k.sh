# r7k: fp64 merged pass B(c-1) + pass A(c) launches: f64 tests + cost, A/B against SDRGPU_F64_MERGE=0
set -o pipefail
PYTEST_K="f64" bash tools/session.sh r7k testk || exit $?
for k in 1 2; do
  timeout -k 10 300 python tools/f64_cost.py >> gpurun_out/r7k_f64cost_merge.json 2>> gpurun_out/r7k_f64cost.err || exit $?
  SDRGPU_TUNING=1 SDRGPU_F64_MERGE=0 timeout -k 10 300 python tools/f64_cost.py >> gpurun_out/r7k_f64cost_sep.json 2>> gpurun_out/r7k_f64cost.err || exit $?
done
