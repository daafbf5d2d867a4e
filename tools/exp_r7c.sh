# r7c: fp64 one-pass 64k kernel (fft64_1p_kernel): parity tests, cost vs the two passes (SDRGPU_F64_1P=0)
set -o pipefail
R=$PWD
PYTEST_K="f64" bash tools/session.sh r7c testk || exit $?
for v in 1 0 1 0; do
  SDRGPU_TUNING=1 SDRGPU_F64_1P=$v timeout -k 10 300 python tools/f64_cost.py > gpurun_out/r7c_f64cost_$v.json 2>> gpurun_out/r7c_f64cost.err || exit $?
done
