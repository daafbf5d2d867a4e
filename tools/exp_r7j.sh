# r7j: fp64 pass A's four-step twiddle recurrence at every size: f64 tests + cost + kernel trace
set -o pipefail
PYTEST_K="f64" bash tools/session.sh r7j testk || exit $?
for k in 1 2; do timeout -k 10 300 python tools/f64_cost.py >> gpurun_out/r7j_f64cost.json 2>> gpurun_out/r7j_f64cost.err || exit $?; done
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r7j_prof -o run -- python3 $GRAFT_REPO_ROOT/tools/f64_cost.py > $GRAFT_REPO_ROOT/gpurun_out/r7j_prof.json 2>&1
