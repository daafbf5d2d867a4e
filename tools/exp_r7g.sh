# r7g: fp64 passes: table log (zdb) + the 64k pass A's four-step twiddle recurrence: f64 parity tests + cost
set -o pipefail
PYTEST_K="f64" bash tools/session.sh r7g testk || exit $?
timeout -k 10 300 python tools/f64_cost.py > gpurun_out/r7g_f64cost.json 2> gpurun_out/r7g_f64cost.err || exit $?
timeout -k 10 300 python tools/f64_cost.py >> gpurun_out/r7g_f64cost.json 2>> gpurun_out/r7g_f64cost.err || exit $?
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r7g_prof -o run -- python3 $GRAFT_REPO_ROOT/tools/f64_cost.py > $GRAFT_REPO_ROOT/gpurun_out/r7g_prof.json 2>&1
