# r7i: persistent fp64 passes (next tile's loads in flight): f64 tests + cost + kernel trace
set -o pipefail
PYTEST_K="f64" bash tools/session.sh r7i testk || exit $?
for k in 1 2; do timeout -k 10 300 python tools/f64_cost.py >> gpurun_out/r7i_f64cost.json 2>> gpurun_out/r7i_f64cost.err || exit $?; done
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r7i_prof -o run -- python3 $GRAFT_REPO_ROOT/tools/f64_cost.py > $GRAFT_REPO_ROOT/gpurun_out/r7i_prof.json 2>&1
