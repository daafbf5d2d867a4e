# r6e: SQ counter sets for the C2 passes and the C5 one-pass kernel (VERDICT r4 items 1-2 evidence)
set -o pipefail
R=$PWD
bash tools/pmc_sets.sh r6e_sq_c2 "fft_pass[AB]_1m_kernel" "$R/bench.py" --config c2 --no-sub --no-cpu --no-ulp --steps 3 --warmup 1 || exit $?
bash tools/pmc_sets.sh r6e_sq_c5 "fft_1p_kernel" "$R/bench.py" --config c5 --no-sub --no-cpu --no-ulp --steps 3 --warmup 1 || exit $?
