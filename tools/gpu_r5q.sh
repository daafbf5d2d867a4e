# r5q: the VFO's later stages as per-stage launches (SDRGPU_VFO_TAIL=0): per-kernel C5 trace
set -o pipefail
OUT=gpurun_out
cd /tmp && export TMPDIR=/tmp
SDRGPU_TUNING=1 SDRGPU_VFO_TAIL=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/r5q_prof" -o run -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --config c5 --no-sub --no-cpu --no-ulp --steps 10 --warmup 2 > "$GRAFT_REPO_ROOT/gpurun_out/r5q_prof.json" 2> "$GRAFT_REPO_ROOT/gpurun_out/r5q_prof.err"
